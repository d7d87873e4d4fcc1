R=$(pwd)
for lib in $R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so $R/_ab/libselunet_nostore.so $R/_ab/libselunet_d2.so $R/selectivenet_for_semantic_segmentation_binary_amd/libselunet.so $R/_ab/libselunet_nostore.so $R/_ab/libselunet_d2.so; do
  echo "== $(basename $lib)"
  SELUNET_LIB=$lib timeout -k 5 90 python3 tools/convt_bench.py --x2 || exit $?
done
