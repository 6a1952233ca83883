cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out
for spec in "opp 128" "opp 256" "opp 512" "vbp_bf 256" "vbp_bf 512" "vbp_bf 1024" "ca_bf 512" "ca_bf 1024"; do
  set -- $spec
  timeout -k 10 200 python -u bench.py --mode $1 --window $2 --steps 3 --warmup 1 --cpu-baseline-seconds 0 > gpurun_out/sw_$1_$2.log 2>&1 || exit $?
done
