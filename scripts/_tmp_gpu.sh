bash scripts/gpu_dram_check.sh dr6 || exit 1
for n in 128 299; do TCI_LIB=build/ab/libtci_chainprof.so timeout -k 10 60 python scripts/dram_time.py 20000 fused 20 $n || exit 1; done
