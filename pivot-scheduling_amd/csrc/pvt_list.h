// pvt_list.h — per-task candidate lists held by one wave (lane j: entry j), shared by the
// streaming score kernel (pvt_kernels.hip) and the band score kernel (pvt_band.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pvt_device.h"
#include "pvt_kernels.h"

namespace pvt {

// Merge a block's candidates (the lanes of pm: each beats entry KL-1, ids distinct from the
// list's) into the wave-held sorted list in one step. Every entry moves down by the number of
// candidates ahead of it; a candidate lands at (entries ahead) + (candidates ahead); whatever
// lands at KL or beyond falls off. Keys are (score bits, tiebreak:id), all distinct, and the
// loop over candidates carries no dependence from one candidate to the next (one insertion
// after another did: each waited for the previous shift and the new last entry).
__device__ __forceinline__ void list_merge(double& s, uint32_t& t, int32_t& i, double cs,
                                           uint32_t ct, int32_t ci, uint64_t pm, uint64_t* m1,
                                           uint64_t* m2) {
  const int lane = lane_id();
  const uint64_t e1 = (uint64_t)__double_as_longlong(s), e2 = ((uint64_t)t << 32) | (uint32_t)i;
  const uint64_t c1 = (uint64_t)__double_as_longlong(cs), c2 = ((uint64_t)ct << 32) | (uint32_t)ci;
  const bool cand = (pm >> lane) & 1ull;
  int below = 0, mypos = KL;
  for (uint64_t q = pm; q; q &= q - 1) {
    const int L = __builtin_ctzll(q);
    const uint64_t x1 = readlane_u64(c1, L), x2 = readlane_u64(c2, L);
    const bool elt = (e1 < x1) | ((e1 == x1) & (e2 < x2));     // entry ahead of candidate L
    const bool clt = cand & ((c1 < x1) | ((c1 == x1) & (c2 < x2)));
    below += elt ? 0 : 1;
    const int pos = __popcll(__ballot(elt)) + __popcll(__ballot(clt));
    mypos = (lane == L) ? pos : mypos;
  }
  const int np = lane + below;
#ifdef PVT_BAND_CHECK
  // diagnostic: every slot must be written before it is read (no real entry has id 0xdeadbeef)
  m1[lane] = 0xdeadbeefdeadbeefull; m2[lane] = 0xdeadbeefdeadbeefull;
  wave_sync();
#endif
  if (np < KL) { m1[np] = e1; m2[np] = e2; }
  if (mypos < KL) { m1[mypos] = c1; m2[mypos] = c2; }
  wave_sync();
  const uint64_t r1 = m1[lane], r2 = m2[lane];
  wave_sync();   // read before the next merge writes
#ifdef PVT_BAND_CHECK
  {
    const uint64_t un = __ballot((uint32_t)r2 == 0xdeadbeefu);
    if (un && lane == 0)
      printf("list_merge: unwritten slots %llx (candidates %llx)\n", (unsigned long long)un,
             (unsigned long long)pm);
  }
#endif
  s = __longlong_as_double((long long)r1);
  t = (uint32_t)(r2 >> 32);
  i = (int32_t)(uint32_t)r2;
}

// Radius on the memory dimension implied by a squared-norm limit: an exact pass (fl(s2) <= lim,
// s2 the FMA chain, every term >= 0, so fl(s2) >= fl(x1*x1)) implies |fl(a1 - d1)| <= rad(lim).
// This one subtract-and-compare rejects nearly every candidate once a task's list has filled
// (the best residuals are small next to the spread of host memory); only survivors pay for the
// four-dimensional fit, the residual norm and the exact limit.
__device__ __forceinline__ double rad(double lim) {
  if (!(lim < DINF)) return DINF;
  if (lim < 0.0) return -1.0;
  return __builtin_sqrt(lim) * (1.0 + 0x1p-40);
}

// The same radius straight from a vbp threshold, without the square root: with
// r = fl(thr (1 + 2^-40)), sqrt(vbp_lim(thr)) <= r (1 + 2^-41 + 2^-52), and fl(r (1 + 2^-38))
// exceeds that with room for the rounding of fl(x1 * x1).
__device__ __forceinline__ double vbp_rad(double thr) {
  if (!(thr < DINF)) return DINF;
  return (thr * (1.0 + 0x1p-40)) * (1.0 + 0x1p-38);
}

}  // namespace pvt
