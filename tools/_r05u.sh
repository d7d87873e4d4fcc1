cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
B="python3 $R/bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-kernel-timing --no-full-loop --no-bf16 --no-exact --no-size512 --no-input-loop"
mkdir -p $R/gpurun_out/r05u
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05u/r1 -o p -- $B > $R/gpurun_out/r05u/r1.log 2>&1 &&
SELUNET_BN_FLAG_RATIO=1e9 timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05u/rinf -o p -- $B > $R/gpurun_out/r05u/rinf.log 2>&1
echo rc=$?
