set -e
mkdir -p gpurun_out/ck2
timeout -k 10 200 python -u -m pytest tests/test_gpu_ckpt.py tests/test_gpu_federation.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ck2/test.log 2>&1
B="timeout -k 10 150 python bench.py --steps 10 --warmup 3 --clients 1"
$B > gpurun_out/ck2/c1_ckpt.log 2>&1
$B --no-ckpt > gpurun_out/ck2/c1_nockpt.log 2>&1
$B > gpurun_out/ck2/c1_ckpt2.log 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > gpurun_out/ck2/c8.log 2>&1
echo done
