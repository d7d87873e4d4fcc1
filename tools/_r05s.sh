R=$(pwd)
for lib in $R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so $R/_ab/libselunet_he64.so $R/_ab/libselunet_heall.so $R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so $R/_ab/libselunet_he64.so $R/_ab/libselunet_heall.so; do
  echo "== $(basename $lib)"
  SELUNET_LIB=$lib timeout -k 5 120 python3 tools/conv_bench.py --dtype fp32 --x2 --iters 10 --only fwd --layers enc2_2,dec3_1,bot4_1,dec1_2 || exit $?
  SELUNET_LIB=$lib timeout -k 5 120 python3 tools/conv_bench.py --dtype fp32 --x2 --iters 10 --only dgrad --layers enc1_2,dec1_1,enc2_2,dec3_1 || exit $?
done
