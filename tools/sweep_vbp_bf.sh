# vbp best-fit config-5 sweep: window sizes x band list segments (PVT_BAND_SEGS), parity checked
for w in 512 1024; do for sg in 16; do
PVT_BAND_SEGS=$sg timeout -k 10 120 python bench.py --mode vbp_bf --window $w --extra 0 --replay 0 --cpu-baseline-seconds 0 > gpurun_out/sw_${w}_${sg}.log 2>&1 || exit 1
tail -1 gpurun_out/sw_${w}_${sg}.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('w=$w S=$sg', round(d['ms_per_step'],3), d['parity'], {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()}, d.get('windows_per_step'), d.get('refills_per_step'))"
done; done
