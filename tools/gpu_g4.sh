tools/gpu_step.sh st_lw 150 python tools/lwalk_stamps.py 1000000 10000 && \
tools/gpu_step.sh st_opp 150 python tools/commit_stamps.py 2 1000000 10000 && \
tools/gpu_step.sh b_vbpbf 200 python bench.py --mode vbp_bf --extra 0 --replay 0 --cpu-baseline-seconds 0 && \
tools/gpu_step.sh b_opp 200 python bench.py --mode opp --extra 0 --replay 0 --cpu-baseline-seconds 0
