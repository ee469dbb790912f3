# Round-4 check of the row-coalesced framebuffer stores in k_inw_pm: INW parity + exactness on
# the default build, A/B against the previous kernels (librt_hip_prev.so), WRITE_SIZE of both.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r04_rows; rm -rf $O; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bvh_exact.py -k "inw" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/gate.log 2>&1 || { echo GATE_FAILED; tail -20 $O/gate.log; exit 1; }
tail -1 $O/gate.log
NOPARITY=1 STEPS=5 bash tools/gpu/ab.sh c3 "- _prev" || exit 1
for v in "" _prev; do
  RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip$v.so timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_w$v -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_w$v.log 2>&1 || exit 1
done
python3 - $O <<'PY'
import csv, glob, sys, collections, os
for d in sorted(glob.glob(sys.argv[1] + "/pmc_w*")):
    if not os.path.isdir(d): continue
    agg = collections.defaultdict(float)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_inw_pm" in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
    print(os.path.basename(d), {k: round(v * 1024 / 2 / 1e9, 4) for k, v in agg.items()}, "GB per frame")
PY
RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_occ.so timeout -k 10 200 python3 tools/inw_occ.py c5 64 > $O/occ_c5.json 2> $O/occ_c5.err || exit 1
RT_HIP_LIB=$GRAFT_REPO_ROOT/raytracing-tests_amd/librt_hip_occ.so timeout -k 10 200 python3 tools/inw_occ.py c3 > $O/occ_c3.json 2> $O/occ_c3.err || exit 1
