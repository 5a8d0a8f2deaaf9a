# Build library variants for A/B runs: canu_amd/lib/ab_<name>.so from the current sources
# with extra -D flags.   usage: bash tools/build_ab.sh name "-DFOO=1 -DBAR=2" [name2 "flags2" ...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
while [ $# -ge 2 ]; do
  n=$1; f=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off $f \
    -o $R/canu_amd/lib/ab_$n.so $R/canu_amd/csrc/ovl_api.hip &
done
wait
ls -la $R/canu_amd/lib/ab_*.so
