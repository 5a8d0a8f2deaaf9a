set -o pipefail
mkdir -p gpurun_out
for v in base SALU VALU; do
 if [ $v = base ]; then L=$PWD/canu_amd/lib/libcanu_ovl.so; else L=$PWD/canu_amd/lib/libcanu_ovl_pad$v.so; fi
 CANU_OVL_LIB=$L timeout -k 10 300 python bench.py --reads 10000 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/pad_$v.log 2>&1 || exit 1
 echo $v $(grep -o '"extend": [0-9.]*' gpurun_out/pad_$v.log)
done
