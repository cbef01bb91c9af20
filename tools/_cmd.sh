mkdir -p gpurun_out
bash tools/ab.sh 3 fw8=opencv_amd/lib/libtbdk.so fw16=opencv_amd/lib/libtbdk_fw16.so fw4=opencv_amd/lib/libtbdk_fw4.so || exit 1
