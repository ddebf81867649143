#!/bin/bash
# A/B build of libawq_hip.so with extra compile flags on ONE source file (the others from
# the product build): bash scripts/build_variant.sh <name> <source.hip> <flags...>
#   -> awq-converter_amd/awq_quantizer/_lib/ab/libawq_hip_<name>.so (travels with gpurun;
#      scripts/generic_bench.py --lib loads it)
set -eu
NAME=$1; SRC=$2; shift 2
cd "$(dirname "$0")/../awq-converter_amd/csrc"
make -s all
mkdir -p build/ab_$NAME ../awq_quantizer/_lib/ab
HIPFLAGS="-O3 --offload-arch=gfx950 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math -fhip-fp32-correctly-rounded-divide-sqrt"
/opt/rocm/bin/hipcc $HIPFLAGS "$@" -Rpass-analysis=kernel-resource-usage -c $SRC -o build/ab_$NAME/${SRC%.hip}.o 2> build/ab_$NAME/remarks.txt
OBJS=""
for src in awq_capi awq_fast awq_rowgroup awq_generic awq_export awq_actsearch awq_stream awq_ptfile; do
  o=build/$src.o; b=$src.o
  if [ "$b" = "${SRC%.hip}.o" ]; then OBJS="$OBJS build/ab_$NAME/$b"; else OBJS="$OBJS $o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o ../awq_quantizer/_lib/ab/libawq_hip_$NAME.so $OBJS
echo "built _lib/ab/libawq_hip_$NAME.so"
