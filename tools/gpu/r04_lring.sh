# Round-4 A/B: the k_inw_pm fold ring in LDS (RT_INW_LRING: 128 entries per wave after 120 staged
# nodes) against the global ring; parity gate first, then frames and PMC HBM bytes per frame.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_lring; rm -rf $O; mkdir -p $O
L=$GRAFT_REPO_ROOT/raytracing-tests_amd
V=${VARIANTS:-lring}
G=${GATE:-$V}
for v in $G; do
  RT_HIP_LIB=$L/librt_hip_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py -k "inw" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gate_$v.log 2>&1 || { echo GATE_${v}_FAILED; tail -5 $O/gate_$v.log; exit 1; }
done
A="--steps 5 --warmup 1 --no-cpu-baseline"
for pass in 1 2; do
  for v in base r128 $V; do
    LIB=$L/librt_hip.so; X=""
    case $v in base) ;; r128) X="--opt inw_ring_pm=128";; *) LIB=$L/librt_hip_$v.so;; esac
    RT_HIP_LIB=$LIB timeout -k 10 200 python3 bench.py $A $X > $O/b_${v}_p$pass.json 2> $O/b_${v}_p$pass.err || exit 1
  done
done
for v in ${PMCV:-$V}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    RT_HIP_LIB=$L/librt_hip_$v.so timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc_${v}_$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_${v}_$c.log 2>&1 || exit 1
  done
done
python3 - $O <<'PY'
import json, glob, sys, os, csv, collections
o = sys.argv[1]
for f in sorted(glob.glob(o + "/b_*.json")):
    b = json.load(open(f))
    print(os.path.basename(f), b["ms_per_step"], b["roofline"]["avg_launch_ms"], b["parity"]["exact_frac"] if b.get("parity") else None)
for d in sorted(glob.glob(o + "/pmc_*_*")):
    if not os.path.isdir(d):
        continue
    agg = collections.defaultdict(float)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_inw_pm" in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(os.path.basename(d), {k: round(v * 1024 / 2 / 1e9, 3) for k, v in agg.items()}, "GB per frame (KiB x 1024 / 2 frames, FETCH not doubled)")
PY
