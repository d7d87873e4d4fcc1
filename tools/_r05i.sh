R=$(pwd)
for lib in $R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so $R/_ab/libselunet_nobar.so $R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so $R/_ab/libselunet_nobar.so; do
  echo "== $(basename $lib)"
  SELUNET_LIB=$lib timeout -k 5 120 python3 tools/conv_bench.py --dtype fp32 --x2 --iters 10 --only fwd --layers enc2_2,dec3_1,bot4_1,dec1_2,enc1_2 || exit $?
done
