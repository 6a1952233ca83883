tools/gpu_step.sh t_vbp 400 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_gpu_epochs.py -m gpu -x -q --timeout 200 --timeout-method thread && \
bash tools/gpu_g6.sh
