# Round-4 checks: INW parity + exactness on the default build and on each variant in GATE
# (librt_hip_<v>.so), A/B frames (default, the previous kernels librt_hip_prev.so, the variants),
# PMC FETCH / WRITE of the main kernel per library, lane occupancy at C3 and C5.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_rows; rm -rf $O; mkdir -p $O
L=$GRAFT_REPO_ROOT/raytracing-tests_amd
G=${GATE:-"park hyb1024 hyb512"}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py -k "inw" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gate.log 2>&1 || { echo GATE_FAILED; tail -20 $O/gate.log; exit 1; }
tail -1 $O/gate.log
for v in $G; do
  RT_HIP_LIB=$L/librt_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py -k "inw" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gate_$v.log 2>&1 || { echo GATE_${v}_FAILED; tail -20 $O/gate_$v.log; exit 1; }
  tail -1 $O/gate_$v.log
done
V="- _prev"; for v in $G; do V="$V _$v"; done
NOPARITY=1 STEPS=5 bash tools/gpu/ab.sh c3 "$V" || exit 1
for v in "" _prev $(for x in $G; do echo _$x; done); do
  for c in FETCH_SIZE WRITE_SIZE; do
    RT_HIP_LIB=$L/librt_hip$v.so timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc${v:-_default}_$c -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc${v:-_default}_$c.log 2>&1 || exit 1
  done
done
python3 - $O <<'PY'
import csv, glob, sys, collections, os
for d in sorted(glob.glob(sys.argv[1] + "/pmc_*")):
    if not os.path.isdir(d): continue
    agg = collections.defaultdict(float)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_inw_pm" in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(os.path.basename(d), {k: round(v * 1024 / 2 / 1e9, 4) for k, v in agg.items()}, "GB per frame (FETCH not doubled)")
PY
RT_HIP_LIB=$L/librt_hip_occ.so timeout -k 10 200 python3 tools/inw_occ.py c5 64 > $O/occ_c5.json 2> $O/occ_c5.err || exit 1
RT_HIP_LIB=$L/librt_hip_occ.so timeout -k 10 200 python3 tools/inw_occ.py c3 > $O/occ_c3.json 2> $O/occ_c3.err || exit 1
