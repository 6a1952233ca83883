tools/gpu_step.sh t_vbp 400 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 200 --timeout-method thread -k "vbp or VBP or band or headline or config5" && \
tools/gpu_step.sh st_lw 150 python tools/lwalk_stamps.py 1000000 10000 && \
tools/gpu_step.sh b_vbpbf 200 python bench.py --mode vbp_bf --extra 0 --replay 0 --cpu-baseline-seconds 0
