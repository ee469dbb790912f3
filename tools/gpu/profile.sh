# Round-end evidence, part 2: the bench line of one config, rocprofv3 kernel trace of the same
# command, and PMC passes (one counter group per pass), summed for the main kernel into
# gpurun_out/prof_<cfg>/pmc_<cfg>.json (copy to profiles/ to make bench.py report roofline.traffic).
#   gpurun -- 'bash tools/gpu/profile.sh c3'        (c3 | c2 | c5 | ns; STEPS=k for the bench line;
#   BENCH_ARGS="--opt inw_qnodes=1" TAG=c3_gq: extra bench arguments, output under prof_<TAG>)
set -o pipefail
CFG=${1:-c3}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd "$R"
TAG=${TAG:-$CFG}
X=${BENCH_ARGS:-}
O=gpurun_out/prof_$TAG
rm -rf $O && mkdir -p $O
timeout -k 10 500 python3 bench.py --config $CFG --steps ${STEPS:-10} $X > $O/bench.json 2> $O/bench.err || exit 1
ARGS="--config $CFG --steps 1 --warmup 1 --no-cpu-baseline $X"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py $ARGS > $O/kt.log 2>&1 || exit 1
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 400 rocprofv3 --pmc $grp -d $O/pmc$i -o run --output-format csv -- python3 bench.py $ARGS > $O/pmc$i.log 2>&1 || exit 1
done
python3 - "$O" "$CFG" <<'PY' || exit 1
import json, subprocess, sys
o, cfg = sys.argv[1], sys.argv[2]
b = json.load(open(f"{o}/bench.json"))
k, c = b["roofline"]["kernel"], b["config"]
subprocess.run([sys.executable, "tools/pmc_summary.py", "--dir", o, "--kernel", k, "--config", str(c["width"]),
                str(c["height"]), str(c["spp"]), "--launches-per-frame", str(b["roofline"]["launches_per_frame"]),
                "--frames", "2", "--out", f"{o}/pmc_{cfg}.json"], check=True, stdout=subprocess.DEVNULL)
PY
