tools/gpu_step.sh t_all 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread && \
bash tools/gpu_g6.sh
