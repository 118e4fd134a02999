set -e
mkdir -p gpurun_out/ab2
B="timeout -k 10 150 python bench.py --steps 10 --warmup 3"
$B --clients 1 > gpurun_out/ab2/c1_def.log 2>&1
BCFL_LINEAR_PERSIST=0 $B --clients 1 > gpurun_out/ab2/c1_nopersist.log 2>&1
$B --clients 1 --overlap-wgrad 0 > gpurun_out/ab2/c1_noov.log 2>&1
BCFL_LINEAR_PERSIST=0 $B --clients 1 --overlap-wgrad 0 > gpurun_out/ab2/c1_nopersist_noov.log 2>&1
$B > gpurun_out/ab2/c8_def.log 2>&1
BCFL_LINEAR_PERSIST=0 $B > gpurun_out/ab2/c8_nopersist.log 2>&1
$B --clients 1 > gpurun_out/ab2/c1_def2.log 2>&1
BCFL_LINEAR_PERSIST=0 $B --clients 1 > gpurun_out/ab2/c1_nopersist2.log 2>&1
echo done
