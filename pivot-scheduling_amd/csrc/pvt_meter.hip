// pvt_meter.hip — Meter aggregates of a batch of scenarios (SURVEY.md §8(f) rank 4;
// reference resources/meter.py:31-53, resources/__init__.py:565-569).
//
// One 256-thread workgroup per scenario, in the reference's nesting: per host the sum of its
// intervals (a thread per host, intervals in order); per route (a wave per route, lanes over
// its packets so the packet / transfer arrays stream coalesced) the sum of its packets' transfer
// sizes, then cost * size / 8000; the block sums the partials in a fixed tree. Only the order
// across hosts, across a route's packets and across routes differs from the reference's
// left-to-right sums (fp64; the north star's 1e-9 relative bound holds by a wide margin: all
// terms are non-negative). HBM-bound streaming reduction, no MFMA.
#include <hip/hip_runtime.h>

#include "pvt_meter.h"

namespace pvt {

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = red[0];
#pragma unroll
  for (int w = 1; w < MET_THREADS / 64; ++w) s += red[w];
  return s;
}

__device__ __forceinline__ bool range_ok(const int64_t* off, int64_t i, int64_t rows,
                                         int64_t n, int64_t* lo, int64_t* hi) {
  if (i < 0 || i >= rows) return false;
  *lo = off[i];
  *hi = off[i + 1];
  return *lo >= 0 && *hi >= *lo && *hi <= n;
}

__global__ void __launch_bounds__(MET_THREADS) meter_kernel(MeterArgs a) {
  __shared__ double red[MET_THREADS / 64];
  const int s = blockIdx.x;
  bool ok = true;
  // cumulative_instance_hours: sum over hosts of sum over intervals of (end - start), / 3600
  double hours = 0.0;
  int64_t h0, h1;
  if (range_ok(a.host_off, s, a.n_scen, a.n_host_rows, &h0, &h1)) {
    for (int64_t h = h0 + threadIdx.x; h < h1; h += MET_THREADS) {
      int64_t v0, v1;
      if (!range_ok(a.iv_off, h, a.n_host_rows, a.n_iv, &v0, &v1)) { ok = false; continue; }
      double acc = 0.0;
      for (int64_t v = v0; v < v1; ++v) acc += a.iv_end[v] - a.iv_start[v];
      hours += acc;
    }
  } else {
    ok = false;
  }
  // total_network_traffic_cost and average_congestion_delay: one wave per route, lanes over
  // its packets (coalesced), each lane folding its packet's transfers in order
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double cost = 0.0, delay = 0.0, npk = 0.0;
  int64_t r0, r1;
  if (range_ok(a.route_off, s, a.n_scen, a.n_routes, &r0, &r1)) {
    for (int64_t r = r0 + wave; r < r1; r += MET_THREADS / 64) {
      int64_t p0, p1;
      if (!range_ok(a.pkt_off, r, a.n_routes, a.n_pkts, &p0, &p1)) { ok = false; continue; }
      double size = 0.0, dl = 0.0;
      for (int64_t p = p0 + lane; p < p1; p += 64) {
        int64_t t0, t1;
        if (!range_ok(a.tr_off, p, a.n_pkts, a.n_tr, &t0, &t1)) { ok = false; continue; }
        double ps = 0.0;
        for (int64_t t = t0; t < t1; ++t) {
          ps += a.tr_size[t];
          if (t > t0) dl += a.tr_start[t] - a.tr_end[t - 1];
        }
        size += ps;
      }
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) {
        size += __shfl_xor(size, o, 64);
        dl += __shfl_xor(dl, o, 64);
      }
      if (lane == 0) {
        cost += a.route_cost[r] * size / 8000.0;
        delay += dl;
        npk += (double)(p1 - p0);
      }
    }
  } else {
    ok = false;
  }
  hours = block_sum(hours, red);
  cost = block_sum(cost, red);
  delay = block_sum(delay, red);
  npk = block_sum(npk, red);
  if (!ok) atomicAdd(a.bad, 1);
  if (threadIdx.x == 0) {
    a.instance_hours[s] = hours / 3600.0;
    a.egress_cost[s] = cost;
    a.congestion_delay[s] = npk > 0.0 ? delay / npk : 0.0;
  }
}

void launch_meter(const MeterArgs& a, hipStream_t st) {
  if (a.n_scen <= 0) return;
  meter_kernel<<<a.n_scen, MET_THREADS, 0, st>>>(a);
}

}  // namespace pvt
