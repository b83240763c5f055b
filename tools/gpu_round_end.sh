# Round-end GPU artifacts: the GPU test suite, smoke, the C3 bench line and its
# kernel-trace stats, the C5 frame, and a two-rank gloo rehearsal (auto split).
# Usage: bash tools/gpu_round_end.sh TAG   (outputs under gpurun_out/TAG/)
set -u
T=${1:-r04z}
D=gpurun_out/$T
mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python -u bench.py > $D/bench_C3.json 2> $D/bench_C3.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof_C3 -o run -- python bench.py --cpu-seconds 0 > $D/bench_C3_prof.json 2> $D/bench_C3_prof.err || { echo "rocprof failed"; exit 1; }
timeout -k 10 300 python -u bench.py --scene O --size 8192 --max-steps 512 --steps 5 --warmup 1 --cpu-seconds 0 > $D/bench_C5.json 2> $D/bench_C5.err || { echo "C5 failed"; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 5 --warmup 1 --cpu-seconds 0 > $D/bench_n2_gloo.json 2> $D/bench_n2_gloo.err || { echo "gloo n2 failed"; exit 1; }
echo round-end done
