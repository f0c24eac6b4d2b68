set -o pipefail
mkdir -p gpurun_out
( nproc; cat /sys/fs/cgroup/cpu.max; python3 -c 'import os; print(len(os.sched_getaffinity(0)), os.cpu_count())'; free -g ) > gpurun_out/probe.txt 2>&1
timeout -k 10 900 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
echo rc=$?
