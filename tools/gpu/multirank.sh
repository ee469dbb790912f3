# Multi-rank rehearsal on one GPU (gloo collectives, shared device): the frames assembled from
# 1, 2 and 3 ranks must be bit-identical.
#   gpurun -- 'bash tools/gpu/multirank.sh c3 [bench args for the multi-rank runs, e.g. --balance-time]'
set -o pipefail
CFG=${1:-c3}
shift 1 2>/dev/null
X="$*"
O=gpurun_out/multirank_$CFG
rm -rf $O && mkdir -p $O
A="--config $CFG --steps 1 --warmup 1 --no-cpu-baseline --spp 8"
timeout -k 10 300 python bench.py $A --save-image $O/f1.npy > $O/n1.json 2> $O/err.log || exit 1
for n in 2 3; do
  RT_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29510 + n)) bench.py --gpus $n $A $X --save-image $O/f$n.npy > $O/n$n.json 2>> $O/err.log || exit 1
done
python -c "
import numpy as np
a = np.load('$O/f1.npy')
import os
da = np.load('$O/f1.depth.npy') if os.path.exists('$O/f1.depth.npy') else None
for n in (2, 3):
    b = np.load('$O/f%d.npy' % n)
    line = 'ranks %d bit-identical to 1 rank: %s %s' % (n, np.array_equal(a.view(np.uint32), b.view(np.uint32)), a.shape)
    if da is not None:
        db = np.load('$O/f%d.depth.npy' % n)
        line += ' depth: %s' % np.array_equal(da.view(np.uint32), db.view(np.uint32))
    print(line)
" | tee $O/check.txt
rm -f $O/f*.npy  # frames are 33 MB each: keep gpurun_out under its copy-back limit
