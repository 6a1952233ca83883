// pvt_zwin_dev.h -- the frontier walk's window compaction (device code), shared by the walk
// (pvt_zwalk.hip, 256 threads) and the grouped order's launch, which prebuilds the windows of a
// round's first epoch (pvt_kernels.hip, 1024 threads).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pvt_device.h"

namespace pvt {

// The first WM hosts of [h_lo, h_hi), in index order, whose zone is in the mask U, appended
// to wid / wz from *nwin on: passes of SCAN rows x NT threads x 4 hosts (one 16-byte zone
// load per thread and row, every load of a pass in flight at once, the next pass's issued before
// this one is compacted), a stable block compaction (per row: a DPP scan of the threads' hit
// counts, the waves' totals through LDS); the block stops at the pass that fills the window.
template <int WM, int NT, int SCAN>
__device__ __forceinline__ void compact_zone_window_t(const int32_t* zone, int Z, uint32_t U,
                                                      int h_lo, int h_hi, int32_t* wid, int32_t* wz,
                                                      int32_t (*cnt)[NT / 64], int32_t* nwin) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int SPAN = SCAN * NT * 4;
  const int a_lo = h_lo & ~3;
  // (16-byte loads need a 16-byte aligned zone array: a caller's offset pointer takes the
  // element loads, as does the last partial quad)
  const bool vec = ((uintptr_t)zone & 15) == 0;
  auto load = [&](int hb) -> int4 {
    if (vec && hb + 4 <= h_hi) return *reinterpret_cast<const int4*>(zone + hb);
    int4 r;
    r.x = hb < h_hi ? zone[hb] : -1;
    r.y = hb + 1 < h_hi ? zone[hb + 1] : -1;
    r.z = hb + 2 < h_hi ? zone[hb + 2] : -1;
    r.w = hb + 3 < h_hi ? zone[hb + 3] : -1;
    return r;
  };
  int4 zz[SCAN];
#pragma unroll
  for (int k = 0; k < SCAN; k++) zz[k] = load(a_lo + (k * NT + tid) * 4);
  for (int h0 = a_lo; h0 < h_hi; h0 += SPAN) {
    const int have = *nwin;
    if (have >= WM) break;
    int4 zn[SCAN];                        // the next pass's zones, in flight during this one
    if (h0 + SPAN < h_hi) {
#pragma unroll
      for (int k = 0; k < SCAN; k++) zn[k] = load(h0 + SPAN + (k * NT + tid) * 4);
    }
    uint32_t hm[SCAN];                    // per row: bit c = host hb + c is a window host
    int ex[SCAN];                         //   its hits before this thread's, in the wave
#pragma unroll
    for (int k = 0; k < SCAN; k++) {
      const int hb = h0 + (k * NT + tid) * 4;
      const int zc[4] = {zz[k].x, zz[k].y, zz[k].z, zz[k].w};
      uint32_t m = 0;
#pragma unroll
      for (int c = 0; c < 4; c++)
        m |= (hb + c >= h_lo && zc[c] >= 0 && zc[c] < Z && ((U >> zc[c]) & 1u)) ? (1u << c) : 0u;
      hm[k] = m;
      const int n = __popc(m);
      const int incl = wave_incl_scan_dpp(n);
      ex[k] = incl - n;
      const int tot = __builtin_amdgcn_readlane(incl, 63);
      if (lane == 0) cnt[k][wave] = tot;
    }
    __syncthreads();
    // every row's counts read before any window store (the stores may alias cnt for the
    // compiler, which then re-read it after each one: a serial LDS chain per pass)
    int before[SCAN], rowtot[SCAN];
#pragma unroll
    for (int k = 0; k < SCAN; k++) {
      int bf = 0, tt = 0;
#pragma unroll
      for (int w = 0; w < (NT / 64); w++) {
        const int c = cnt[k][w];
        bf += (w < wave) ? c : 0;
        tt += c;
      }
      before[k] = bf;
      rowtot[k] = tt;
    }
    int pre = have;
#pragma unroll
    for (int k = 0; k < SCAN; k++) {
      const int hb = h0 + (k * NT + tid) * 4;
      const int zc[4] = {zz[k].x, zz[k].y, zz[k].z, zz[k].w};
      int pos = pre + before[k] + ex[k];
#pragma unroll
      for (int c = 0; c < 4; c++) {
        if ((hm[k] >> c) & 1u) {
          if (pos < WM) {
            wid[pos] = hb + c;
            if (wz) wz[pos] = zc[c];
          }
          pos++;
        }
      }
      pre += rowtot[k];
    }
    __syncthreads();
    if (tid == 0) *nwin = min(pre, WM);
    __syncthreads();
    if (h0 + SPAN < h_hi) {
#pragma unroll
      for (int k = 0; k < SCAN; k++) zz[k] = zn[k];
    }
  }
}


}  // namespace pvt
