mkdir -p gpurun_out; out=gpurun_out/r5_quad2.log; : > $out
for qm in 1 2 3; do echo "== QUADB $qm" >> $out; HYDRA_ATTN8_QUADB=$qm timeout -k 10 120 python -u tools/bench_attn8.py 2560 2311 2>&1 | grep "W=8\|W=6\|W=4" >> $out; done
echo "== QUAD 0" >> $out; HYDRA_ATTN8_QUAD=0 timeout -k 10 120 python -u tools/bench_attn8.py 2560 2311 2>&1 | grep "W=8" >> $out
HYDRA_ATTN8_QUADB=1 timeout -k 10 120 python -u -m pytest -q -x --timeout 60 tests/test_attention8_gpu.py >> $out 2>&1
