// pvt_meter.h — Meter aggregates over a batch of scenarios (see pvt_meter.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pvt {

constexpr int MET_THREADS = 256;

struct MeterArgs {
  int32_t n_scen;
  int64_t n_host_rows, n_iv, n_routes, n_pkts, n_tr;
  const int64_t *host_off, *iv_off, *route_off, *pkt_off, *tr_off;
  const double *iv_start, *iv_end, *route_cost, *tr_start, *tr_end, *tr_size;
  double *instance_hours, *egress_cost, *congestion_delay;
  int32_t* bad;
};

void launch_meter(const MeterArgs& a, hipStream_t st);

}  // namespace pvt
