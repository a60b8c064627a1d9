#!/usr/bin/env bash
# Host-only ASan/UBSan build of the C ABI + the argument driver (CPU host only:
# GPU AddressSanitizer is not available on the pool).  Device code is compiled
# as usual; -Xarch_host puts the sanitizers on the host half only.
#   scripts/san/build_abi_asan.sh && slam-1_amd/build_asan/abi_args
set -euo pipefail
cd "$(dirname "$0")/../.."
OUT=slam-1_amd/build_asan
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN="-Xarch_host -fsanitize=address,undefined -Xarch_host -fno-omit-frame-pointer -Xarch_host -fno-sanitize-recover=undefined"
FLAGS="-O1 -g -std=c++17 --offload-arch=gfx950 -fPIC -ffp-contract=off -munsafe-fp-atomics \
       -fhip-fp32-correctly-rounded-divide-sqrt -mllvm -amdgpu-mfma-vgpr-form -Iinclude"
objs=()
for f in slam-1_amd/csrc/*.hip; do
  o="$OUT/$(basename "${f%.hip}").o"
  if [[ ! -f "$o" || "$f" -nt "$o" || include/slam355.h -nt "$o" ]]; then
    $HIPCC $FLAGS $SAN -c "$f" -o "$o" &
  fi
  objs+=("$o")
done
wait
gcc -O1 -g -std=c11 -Iinclude -fsanitize=address,undefined -fno-omit-frame-pointer \
    -c scripts/san/abi_args.c -o "$OUT/abi_args.o"
$HIPCC --offload-arch=gfx950 -fsanitize=address,undefined -o "$OUT/abi_args" \
    "$OUT/abi_args.o" "${objs[@]}"
echo "built $OUT/abi_args"
