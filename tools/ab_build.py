"""Build an A/B variant of libselunet.so with one source file replaced (profiling tool).

    python tools/ab_build.py NAME csrc_file=/path/to/variant.hip [csrc_file=...]

Compiles the replaced sources for gfx950, links them with the in-tree objects of every other
source (selectivenet_for_semantic_segmentation_binary_amd/_build/*.o, built by build.py) and
writes _ab/libselunet_NAME.so; select it at run time with SELUNET_LIB (tools/ab_run.sh).
"""
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "selectivenet_for_semantic_segmentation_binary_amd")
sys.path.insert(0, REPO)
from selectivenet_for_semantic_segmentation_binary_amd import build as B  # noqa: E402


def main():
    name, repl = sys.argv[1], dict(a.split("=", 1) for a in sys.argv[2:])
    B.build(verbose=False)
    out = os.path.join(REPO, "_ab")
    os.makedirs(out, exist_ok=True)
    objs = []
    for src in B._sources():
        obj = os.path.join(B.BUILD, src.replace(".hip", ".o"))
        if src in repl:
            tmp = os.path.join(B.CSRC, f"_ab_{name}_{src}")
            shutil.copy(repl[src], tmp)  # compiled next to the real sources (same include paths)
            obj = os.path.join(out, f"{name}_{src}.o")
            try:
                r = subprocess.run([B.HIPCC, *B.FLAGS, "-c", tmp, "-o", obj], capture_output=True, text=True)
            finally:
                os.remove(tmp)
            if r.returncode:
                sys.exit(r.stderr[-4000:])
        objs.append(obj)
    objs.append(os.path.join(B.BUILD, "build_id.o"))  # (selunet_build_id: the tree's sources; SELUNET_LIB skips the check)
    lib = os.path.join(out, f"libselunet_{name}.so")
    subprocess.run([B.HIPCC, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *objs, "-o", lib], check=True)
    print(lib)


if __name__ == "__main__":
    main()
