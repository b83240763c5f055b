set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_r01c.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r01c.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_r01c.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --backend gloo --cpu-seconds 0 --size 1024 > gpurun_out/bench_gloo2.json 2> gpurun_out/bench_gloo2.err || { tail -20 gpurun_out/bench_gloo2.err; exit 2; }
cat gpurun_out/bench_gloo2.json
