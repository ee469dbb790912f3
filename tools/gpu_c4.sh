# bench.py --config c4 (BASELINE configs[3]'s LBVH scene): one full-spp line on one GPU, and a
# 2-rank gloo rehearsal whose assembled frame must equal the 1-rank frame bit for bit
set -o pipefail
O=gpurun_out/c4
mkdir -p $O
timeout -k 10 300 python bench.py --config c4 --steps 1 --warmup 1 > $O/bench_c4.json 2> $O/bench_c4.err || exit 1
A="--config c4 --steps 1 --warmup 0 --no-cpu-baseline --spp 8"
timeout -k 10 200 python bench.py $A --save-image $O/c4_1.npy > $O/c4_1.json 2> $O/c4_1.err || exit 1
RT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 $A --save-image $O/c4_2.npy > $O/c4_2.json 2> $O/c4_2.err || exit 1
python -c "
import numpy as np
a=np.load('$O/c4_1.npy'); b=np.load('$O/c4_2.npy')
print('C4 N2 identical', np.array_equal(a.view(np.uint32), b.view(np.uint32)), a.shape)
" > $O/check.txt
