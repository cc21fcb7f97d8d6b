#!/bin/bash
# Host (GPU box or here): phase split of the native PNG decoder on the e2e_png leg's 8
# distinct synthetic 1080p PNGs (bench.py _encode, seed 1234), single thread, 10 reps each:
# inflate (libdeflate) / unfilter / RGB->BGR, and the whole decode_one.  Output:
# gpurun_out/png_split.txt
set -u -o pipefail
mkdir -p gpurun_out /tmp/llfe_png
g++ -O3 -std=c++17 -Iinclude -o /tmp/llfe_png/png_prof tools/debug/png_prof.cpp \
    low_level_feature_extraction_amd/csrc/jpeg_decode.cpp -lz -ldl -lpthread || exit 1
python3 -c "
import sys; sys.path.insert(0, '.')
import bench
for i in range(8):
    open('/tmp/llfe_png/img%d.png' % i, 'wb').write(bench._encode((i, 1080, 1920, 1234, 'PNG')))
" || exit 1
{
    echo "# $(grep -m1 'model name' /proc/cpuinfo | cut -d: -f2) ; one thread, 10 reps per file"
    for i in 0 1 2 3 4 5 6 7; do timeout -k 5 120 /tmp/llfe_png/png_prof /tmp/llfe_png/img$i.png 10 || exit 1; done
} > gpurun_out/png_split.txt
python3 - <<'PY'
import re
t = open('gpurun_out/png_split.txt').read()
rows = re.findall(r'inflate ([\d.]+) ms unfilter ([\d.]+) ms convert ([\d.]+) ms \| decode_one ([\d.]+) ms', t)
v = [[float(x) for x in r] for r in rows]
m = [sum(c) / len(v) for c in zip(*v)]
s = "mean over %d files: inflate %.2f ms (%.0f %%), unfilter %.2f ms (%.0f %%), convert %.2f ms (%.0f %%), decode_one %.2f ms" % (
    len(v), m[0], 100 * m[0] / m[3], m[1], 100 * m[1] / m[3], m[2], 100 * m[2] / m[3], m[3])
open('gpurun_out/png_split.txt', 'a').write(s + "\n")
print(s)
PY
