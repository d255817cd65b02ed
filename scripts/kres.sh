#!/usr/bin/env bash
# Kernel resource usage (VGPRs, AGPRs, SGPRs, scratch, LDS) of the gfx950 code
# object embedded in a hipcc-built object or shared library:
#   scripts/kres.sh FILE [NAME-REGEX]
set -eu
F=$1; PAT=${2:-.}
T=$(mktemp -d /tmp/kres.XXXX)
B=/opt/rocm/lib/llvm/bin
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fb "$F" /dev/null
TGT=$($B/clang-offload-bundler --list --type=o --input=$T/fb | grep gfx950 | head -1)
$B/clang-offload-bundler --unbundle --type=o --input=$T/fb --targets="$TGT" --output=$T/co
$B/llvm-readelf --notes $T/co | python3 -c "
import sys, re
txt = sys.stdin.read()
pat = re.compile(sys.argv[1])
for blk in txt.split('.name:')[1:]:
    name = blk.split('\n', 1)[0].strip()
    if not pat.search(name) or name.endswith('.kd'):
        continue
    def f(k):
        m = re.search(r'\.' + k + r':\s+(\d+)', blk)
        return m.group(1) if m else '-'
    print(f'{name[:100]:100s} vgpr {f(\"vgpr_count\"):>4} agpr {f(\"agpr_count\"):>4} sgpr {f(\"sgpr_count\"):>4} '
          f'scratch {f(\"private_segment_fixed_size\"):>5} lds {f(\"group_segment_fixed_size\"):>6}')
" "$PAT"
rm -rf $T
