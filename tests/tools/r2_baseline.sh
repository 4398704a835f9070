#!/bin/bash
# Round 2 start: the committed round-1 tree on a fresh box -- host facts,
# smoke, C2 bench line, and a rocprofv3 kernel trace of the same bench.
set -o pipefail
export TMPDIR=/tmp
o=gpurun_out/r2base
mkdir -p $o
(nproc; grep -m1 "model name" /proc/cpuinfo; free -g; cat /sys/fs/cgroup/cpu.max 2>/dev/null) > $o/host.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-lossless --steps 48 > $o/bench.json 2> $o/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $o/kt -o run --output-format csv -- python bench.py --no-cpu-baseline --no-lossless --steps 48 > $o/bench_kt.json 2> $o/bench_kt.err || exit 1
