mkdir -p gpurun_out
L=opencv_amd/lib/libtbdk.so
bash tools/ab.sh 3 cur=$L o2=$L,--ctx-option=tbd_early_order=2 dfr=$L,--ctx-option=tbd_la_defer=1 || exit 1
