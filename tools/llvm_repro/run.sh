#!/bin/bash
# the fp64 NaN states under -mllvm -disable-machine-cse are an
# LLVM AMDGPU bug (an unencodable 64-bit SALU literal).  Shows it on the reduced
# reproducer s_mov_b64_literal.hip: the emitted assembly, the assembler's
# rejection, the object's truncated literal, and (with a GPU) wrong results.
set -u
D=$(cd "$(dirname "$0")" && pwd)
T=$(mktemp -d)
LLVM=/opt/rocm/lib/llvm/bin
for v in default nomcse; do
  F=""; [ $v = nomcse ] && F="-mllvm -disable-machine-cse"
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 --offload-device-only -S -o "$T/$v.s" "$D/s_mov_b64_literal.hip" $F 2>/dev/null
  echo "[$v] s_mov_b64 with a 64-bit literal: $(grep -c 's_mov_b64.*0x[0-9a-f]\{9,\}' "$T/$v.s")"
  grep 's_mov_b64.*0x[0-9a-f]\{9,\}' "$T/$v.s" | sed 's/^/    /'
  /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -o "$T/$v" "$D/s_mov_b64_literal.hip" $F 2>/dev/null
done
printf 's_mov_b64 s[0:1], 0x4049000000000000\n' > "$T/lit.s"
echo "[llvm-mc gfx950] $($LLVM/llvm-mc -arch=amdgcn -mcpu=gfx950 -show-encoding "$T/lit.s" 2>&1 | head -1)"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 --offload-device-only -c -o "$T/nomcse.co" "$D/s_mov_b64_literal.hip" -mllvm -disable-machine-cse 2>/dev/null
$LLVM/clang-offload-bundler --unbundle --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input="$T/nomcse.co" --output="$T/nomcse.elf" 2>/dev/null
echo "[object, -disable-machine-cse] the move as encoded:"
$LLVM/llvm-objdump -d --mcpu=gfx950 "$T/nomcse.elf" | grep "s_mov_b64 s\[0:1\]" | sed 's/^/    /'
if [ -e /dev/kfd ]; then
  for v in default nomcse; do echo "[run $v] $(timeout -k 5 60 "$T/$v")"; done
fi
rm -rf "$T"
