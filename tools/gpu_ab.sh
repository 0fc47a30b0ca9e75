#!/bin/bash
# same-box A/B of the wx3 conv: baseline build (tools/native/wino_base_0) vs the working tree
# (wino_ablate_0), alternated three times.
set -u -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
: > gpurun_out/ab.log
for r in 1 2 3; do
  for b in wino_base_0 wino_ablate_0; do
    echo "== $b" >> gpurun_out/ab.log
    timeout -k 10 60 ./tools/native/$b x3 >> gpurun_out/ab.log 2>&1 || exit $?
  done
done
python3 - <<'PY'
import re, collections
cur = None; t = collections.defaultdict(list)
for l in open('gpurun_out/ab.log'):
    if l.startswith('=='): cur = l.split()[1]; continue
    m = re.search(r'hw=(\d+) c=(\d+): ([\d.]+) us', l)
    if m: t[(m.group(1), m.group(2), cur)].append(float(m.group(3)))
for hw, c in sorted({(k[0], k[1]) for k in t}, key=lambda x: (-int(x[0]), -int(x[1]))):
    a, b = t[(hw, c, 'wino_base_0')], t[(hw, c, 'wino_ablate_0')]
    print(f"hw={hw} c={c}: base {min(a):.1f} us  new {min(b):.1f} us  ({100*(min(b)/min(a)-1):+.1f}%)  runs {a} {b}")
PY
