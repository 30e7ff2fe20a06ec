#!/bin/bash
# Per kernel: global/buffer loads vs full memory-counter drains (s_waitcnt vmcnt(0)).
# Many drains relative to loads means the loads are serialised (typically guarded,
# branchy loads).  Usage: tools/isa_waits.sh <obj.o> [kernel-substring]
set -e
B=/opt/rocm/lib/llvm/bin
obj=$1; pat=${2:-}
tmp=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$tmp/fb.bin "$obj"
tgt=$($B/clang-offload-bundler --type=o --input=$tmp/fb.bin --list | grep gfx950 | head -1)
$B/clang-offload-bundler --unbundle --type=o --input=$tmp/fb.bin --targets="$tgt" --output=$tmp/k.co
$B/llvm-objdump -d --no-show-raw-insn $tmp/k.co > $tmp/k.s
awk -v pat="$pat" '
  /^[0-9a-f]+ <.*>:$/ { name=$2; next }
  { if (pat == "" || index(name, pat) > 0) {
      if ($0 ~ /global_load|buffer_load/) ld[name]++;
      if ($0 ~ /vmcnt\(0\)/) w[name]++;
      seen[name]=1 } }
  END { for (k in seen) printf "%5d loads %5d vmcnt(0)  %s\n", ld[k], w[k], substr(k, 1, 90) }' $tmp/k.s | sort -k3 -rn
rm -rf $tmp
