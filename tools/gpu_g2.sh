tools/gpu_step.sh t_zw 400 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_epochs.py tests/test_gpu_ordered_frontier.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread && \
tools/gpu_step.sh b_cabf 150 python bench.py --extra 0 --replay 0 --cpu-baseline-seconds 0 --steps 20 && \
tools/gpu_step.sh b_vbpff 150 python bench.py --mode vbp_ff --extra 0 --replay 0 --cpu-baseline-seconds 0 && \
tools/gpu_step.sh b_caff 150 python bench.py --mode ca_ff --extra 0 --replay 0 --cpu-baseline-seconds 0 && \
tools/gpu_step.sh st_cabf 120 python tools/zwalk_stamps.py 1000000 10000 libpivot_place_stamps.so ca_bf && \
tools/gpu_step.sh st_vbpff 120 python tools/zwalk_stamps.py 1000000 10000 libpivot_place_stamps.so vbp_ff && \
tools/gpu_step.sh st_caff 120 python tools/zwalk_stamps.py 1000000 10000 libpivot_place_stamps.so ca_ff
