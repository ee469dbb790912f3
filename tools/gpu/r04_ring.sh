# Round-4 A/B on one box: parity gates, bench frames for fold-ring windows and the two-leaf walk
# variant, PMC HBM bytes per ring size, INW lane occupancy, the --rebuild line.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_ring; rm -rf $O; mkdir -p $O
L=$GRAFT_REPO_ROOT/raytracing-tests_amd
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "repeated or inw01_random or update" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gate.log 2>&1 || { echo GATE_FAILED; exit 1; }
for v in pend2 park; do
  RT_HIP_LIB=$L/librt_hip_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py -k "inw" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/gate_$v.log 2>&1 || { echo GATE_${v}_FAILED; exit 1; }
done
A="--steps 5 --warmup 1 --no-cpu-baseline"
for pass in 1 2; do
  for v in base r512 r256 pend2 park park16 park4m8; do
    X=""; LIB=$L/librt_hip.so
    [ $v = r512 ] && X="--opt inw_ring_pm=512"
    [ $v = r256 ] && X="--opt inw_ring_pm=256"
    case $v in pend2|park*) LIB=$L/librt_hip_$v.so;; esac
    RT_HIP_LIB=$LIB timeout -k 10 200 python3 bench.py $A $X > $O/b_${v}_p$pass.json 2> $O/b_${v}_p$pass.err || exit 1
  done
done
for r in 1024 256; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc_${r}_$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --opt inw_ring_pm=$r > $O/pmc_${r}_$c.log 2>&1 || exit 1
  done
done
RT_HIP_LIB=$L/librt_hip_occ.so timeout -k 10 200 python3 tools/inw_occ.py c3 > $O/occ_c3.json 2> $O/occ_c3.err || exit 1
RT_HIP_LIB=$L/librt_hip_occ.so timeout -k 10 200 python3 tools/inw_occ.py c5 64 > $O/occ_c5.json 2> $O/occ_c5.err || exit 1
timeout -k 10 300 python3 bench.py --rebuild --steps 5 --warmup 1 --no-cpu-baseline > $O/rebuild.json 2> $O/rebuild.err || exit 1
python3 - $O <<'PY'
import json, glob, sys, os, csv, collections
o = sys.argv[1]
for f in sorted(glob.glob(o + "/b_*.json")):
    b = json.load(open(f))
    print(os.path.basename(f), b["ms_per_step"], b["roofline"]["avg_launch_ms"], b["path"]["ring_entries"])
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
