#!/bin/bash
# Disassemble the gfx950 code object of one HIP object file: tools/isa_dump.sh OBJ.o OUT.s
set -e
tmp=$(mktemp -d)
/opt/rocm/lib/llvm/bin/llvm-objcopy --dump-section=.hip_fatbin=$tmp/fat.bin "$1"
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$tmp/fat.bin \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$tmp/co.elf
/opt/rocm/lib/llvm/bin/llvm-objdump -d --mcpu=gfx950 $tmp/co.elf > "$2"
rm -rf $tmp
