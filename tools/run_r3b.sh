O=gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py "tests/test_gpu_fullframe.py::test_c2_full_frame_is_the_reference_frame[default]" tests/test_mixture_cap.py > $O/nan1.tests.log 2>&1; echo "tests rc=$?"; tail -2 $O/nan1.tests.log
SRR_LIB=$PWD/simple-raytracing-render_amd/libsrr_slow.so timeout -k 10 300 python tools/slow_rays.py --scene s2 > $O/slow_s2_frame.jsonl 2> $O/slow_s2_frame.err; echo "slow1 rc=$?"; tail -2 $O/slow_s2_frame.err
SRR_LIB=$PWD/simple-raytracing-render_amd/libsrr_slow.so timeout -k 10 300 python tools/slow_rays.py --scene s2 --shards 8 > $O/slow_s2_8.jsonl 2> $O/slow_s2_8.err; echo "slow8 rc=$?"; tail -8 $O/slow_s2_8.err | cut -c1-250
timeout -k 10 300 python tools/shard_balance.py --scene s2 --tile 16 --reps 2 > $O/sb_s2_t16.json 2> $O/sb_s2_t16.err; echo "sb rc=$?"; tail -3 $O/sb_s2_t16.err | cut -c1-300
timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/nan1.bench.log 2>&1; grep -o '"value": [0-9.]*' $O/nan1.bench.log
