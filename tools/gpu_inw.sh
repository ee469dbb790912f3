# INW wide walk: parity / exactness tests of the INW paths, then the INW configs
set -o pipefail
O=gpurun_out/inw
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_textures.py tests/test_gpu_stages.py tests/test_gpu_bvh_exact.py -k "inw or INW or render_matches or textured or stage or golden" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || exit 1
cat $O/configs.jsonl
