set -o pipefail
timeout -k 10 120 python tools/diff_w5.py && CANU_OVL_LIB=$PWD/canu_amd/lib/libcanu_ovl_w5.so timeout -k 10 120 python tools/diff_w5.py
