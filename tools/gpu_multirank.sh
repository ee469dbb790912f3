# multi-rank rehearsal on one GPU: 1 rank vs 2 and 3 ranks (gloo collectives, shared device);
# the assembled frames must be bit-identical
set -o pipefail
mkdir -p gpurun_out
A="--steps 1 --warmup 1 --no-cpu-baseline --spp 8 --balance"  # the timed frame uses the LPT deal
timeout -k 10 300 python bench.py $A --save-image gpurun_out/mr_1.npy > gpurun_out/mr_1.json 2> gpurun_out/mr.err || exit 1
RT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 $A --save-image gpurun_out/mr_2.npy > gpurun_out/mr_2.json 2>> gpurun_out/mr.err || exit 1
RT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 3 $A --save-image gpurun_out/mr_3.npy > gpurun_out/mr_3.json 2>> gpurun_out/mr.err || exit 1
python -c "
import numpy as np
a=np.load('gpurun_out/mr_1.npy'); b=np.load('gpurun_out/mr_2.npy'); c=np.load('gpurun_out/mr_3.npy')
print('N2 identical', np.array_equal(a.view(np.uint32), b.view(np.uint32)), 'N3 identical', np.array_equal(a.view(np.uint32), c.view(np.uint32)), a.shape)
" > gpurun_out/mr_check.txt
