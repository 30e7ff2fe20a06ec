#!/bin/bash
# Disassemble the gfx950 code object inside a hipcc-built .o and count selected
# instructions per kernel.  Usage: tools/isa_stats.sh <obj.o> [kernel-substring] [regex]
set -e
B=/opt/rocm/lib/llvm/bin
obj=$1; pat=${2:-}; re=${3:-'v_pk_fma_f32|v_fmac?_f32|v_exp_f32|ds_read|s_waitcnt|v_mfma'}
tmp=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$tmp/fb.bin "$obj"
$B/clang-offload-bundler --type=o --input=$tmp/fb.bin --list > $tmp/targets
tgt=$(grep gfx950 $tmp/targets | head -1)
$B/clang-offload-bundler --unbundle --type=o --input=$tmp/fb.bin --targets="$tgt" --output=$tmp/k.co
$B/llvm-objdump -d --no-show-raw-insn $tmp/k.co > $tmp/k.s
awk -v pat="$pat" -v re="$re" '
  /^[0-9a-f]+ <.*>:$/ { name=$2; next }
  { if (pat == "" || index(name, pat) > 0) { n[name]++; if (match($0, re)) { split($1, a, " "); c[name, $1]++ ; keys[name]=1 } } }
  END { for (k in n) { printf "%6d insts  %s\n", n[k], substr(k, 1, 100);
        for (kk in c) { split(kk, p, SUBSEP); if (p[1] == k) printf "        %6d %s\n", c[kk], p[2] } } }' $tmp/k.s
rm -rf $tmp
