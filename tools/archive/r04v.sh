# small fp32-output NT/TN GEMMs on gemm3 instead of hipBLASLt: A/B at 64 / 128 / 512 rows
B="python -u bench.py --steps 10 --warmup 3 --no-gen --no-cpu --no-extra"
bash tools/gsteps.sh \
 "300 python -u -m pytest tests/test_gpu_kernels.py -k 'gemm' -q -rf --timeout 120 --timeout-method thread > gpurun_out/r04v_tests.log 2>&1" \
 "240 $B --batch 64 > gpurun_out/r04v_b64.json 2> gpurun_out/r04v_b64.err" \
 "240 SRNN_BLASLT_SMALL_F32=1 $B --batch 64 > gpurun_out/r04v_b64_old.json 2> gpurun_out/r04v_b64_old.err" \
 "240 $B --batch 64 > gpurun_out/r04v_b64b.json 2> gpurun_out/r04v_b64b.err" \
 "240 SRNN_BLASLT_SMALL_F32=1 $B --batch 64 > gpurun_out/r04v_b64_oldb.json 2> gpurun_out/r04v_b64_oldb.err" \
 "240 $B --batch 128 > gpurun_out/r04v_b128.json 2> gpurun_out/r04v_b128.err" \
 "240 SRNN_BLASLT_SMALL_F32=1 $B --batch 128 > gpurun_out/r04v_b128_old.json 2> gpurun_out/r04v_b128_old.err" \
 "240 $B > gpurun_out/r04v_b512.json 2> gpurun_out/r04v_b512.err" \
 "240 SRNN_BLASLT_SMALL_F32=1 $B > gpurun_out/r04v_b512_old.json 2> gpurun_out/r04v_b512_old.err"
