// pvt_batch.hip — resident rounds: one workgroup runs one whole scheduling round with the
// round's hosts held in registers; a launch runs a batch of independent rounds (one per block).
//
// Reference: the same sequential loops as the windowed engine (scheduler/cost_aware.py:84-97,
// :117-127; scheduler/opportunistic.py:11-20; scheduler/vbp.py:19-25, :43-49), visited in the
// reference's order (cost_aware.py:37,60-61 groups + stable sort; vbp.py:17,41). This kernel is
// their direct restatement rather than the snapshot/list formulation: with H <= 4096 hosts a
// round fits in one workgroup's registers (host h lives in thread h / HPL, slot h % HPL, all
// four capacities, its zone, its tiebreak rank and its frozen first-fit key), so every task
// rescans every host at register speed, commits in place, and no state leaves the CU until the
// round ends. It serves
//   - scenario batches (BASELINE config 4): B independent rounds in
//     ONE launch, one block each, so the rounds' sequential walks run side by side on all CUs;
//   - single rounds of the sim.py sizes (100-1000 hosts, configs 1-2) through pvt_place.
//
// Per task (4 waves): each lane reduces its HPL hosts to the best (score bits, tiebreak:host)
// 128-bit key (scores are >= +0, so bit patterns order like values), the wave reduces to its
// minimum, lane 0 posts it in LDS (double-buffered by task parity: ONE barrier per task), and
// every wave picks the same winner from the four posts; the owning thread commits in its
// registers. Opportunistic posts per-wave feasible counts instead; each wave draws the same
// randint(0, n) from its own copy of the MT19937 state (no second barrier), and the wave that
// holds the k-th feasible host commits it.
//
// Numerics as everywhere in the engine: -ffp-contract=off, sequential-FMA squared norms,
// correctly rounded sqrt/div, scores computed in the reference's operation order.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "pivot_place.h"
#include "pvt_device.h"
#include "pvt_kernels.h"
#include "pvt_mt.h"

namespace pvt {

constexpr int RES_WAVES = RES_THREADS / WAVE;
constexpr int RES_CHUNK = 256;           // tasks whose demand rows are staged in LDS at a time
constexpr int RES_MT_STRIDE = 628;       // words per wave-private MT19937 copy (625 used)
constexpr uint64_t NONE = ~0ull;

// Dynamic LDS layout (bytes); the host sizes the launch with the same struct.
struct ResLds {
  int zt, ord, u, cd, ci, mt, slot, total;
  __host__ __device__ ResLds(int Zb, int Tpad) {
    zt = 0;                                            // csum[Zb*Zb], bsum[Zb*Zb] f64
    ord = (16 * Zb * Zb + 15) & ~15;                   // processing order i32[Tpad]
    u = (ord + 4 * Tpad + 15) & ~15;                   // union: sort keys | walk staging
    cd = u;                                            // walk: demand rows f64[CHUNK][4]
    ci = cd + 32 * RES_CHUNK;                          //       anchor, caller, group i32[3][CHUNK]
    mt = ci + 12 * RES_CHUNK;                          //       MT copies u32[WAVES][628]
    slot = mt + 4 * RES_WAVES * RES_MT_STRIDE;         //       posts u64[2][WAVES][2]
    const int walk_end = slot + 32 * RES_WAVES;
    const int sort_end = u + 16 * Tpad;                // sort: u64 ka[Tpad], kb[Tpad]
    total = walk_end > sort_end ? walk_end : sort_end;
  }
};

size_t resident_lds_bytes(int Zb, int Tpad) { return (size_t)ResLds(Zb, Tpad).total; }

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m), hi = __shfl_xor((int)(uint32_t)(v >> 32), m);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t dbits(double x) { return (uint64_t)__double_as_longlong(x); }

// Stable processing order (a2): sort (group, ~bits(||d||2) or 0, caller index) ascending with a
// bitonic network over Tpad entries; the caller index makes every key distinct, so the result
// is the stable order cost_aware.py:37,60-61 / vbp.py:17,41 produce.
__device__ void res_order(const pvt_round& R, bool grouped, bool sorted, uint64_t* ka, uint64_t* kb,
                          int32_t* ord, int Tpad) {
  const int T = R.n_tasks, tid = threadIdx.x;
  for (int i = tid; i < Tpad; i += RES_THREADS) {
    if (i < T) {
      const uint32_t g = grouped ? (uint32_t)R.task_group[i] : 0u;
      ka[i] = ((uint64_t)g << 32) | (uint32_t)i;
      if (sorted) {
        const double n = __builtin_sqrt(norm2_seq(R.dem[i], R.dem[(size_t)T + i],
                                                  R.dem[2 * (size_t)T + i], R.dem[3 * (size_t)T + i]));
        kb[i] = ~dbits(n);                               // descending norm
      } else {
        kb[i] = 0;
      }
    } else {
      ka[i] = NONE;
      kb[i] = NONE;
    }
  }
  __syncthreads();
  if (grouped || sorted) {
    for (int k = 2; k <= Tpad; k <<= 1) {
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int i = tid; i < Tpad; i += RES_THREADS) {
          const int l = i ^ j;
          if (l > i) {
            const uint64_t ai = ka[i], al = ka[l], bi = kb[i], bl = kb[l];
            const uint32_t gi = (uint32_t)(ai >> 32), gl = (uint32_t)(al >> 32);
            const bool less_li = gl < gi || (gl == gi && (bl < bi || (bl == bi && (uint32_t)al < (uint32_t)ai)));
            if (less_li == ((i & k) == 0)) {
              ka[i] = al; ka[l] = ai; kb[i] = bl; kb[l] = bi;
            }
          }
        }
        __syncthreads();
      }
    }
  }
  for (int i = tid; i < T; i += RES_THREADS) ord[i] = (int32_t)(uint32_t)ka[i];
  __syncthreads();
}

template <int MODE, int HPL>
__global__ __launch_bounds__(RES_THREADS) void resident_kernel(ResidentArgs A) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool CA = (MODE == CA_FF || MODE == CA_BF);
  constexpr bool STRICT = (MODE == CA_FF || MODE == VBP_BF);
  const ResLds Lo(A.Zb, A.Tpad);
  const pvt_round R = reinterpret_cast<const pvt_round*>(A.rounds)[blockIdx.x];   // SGPRs
  const int H = R.n_hosts, T = R.n_tasks, Z = R.n_zones;
  const int tid = threadIdx.x, lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  double* csum = reinterpret_cast<double*>(smem + Lo.zt);
  double* bsum = csum + A.Zb * A.Zb;
  int32_t* ord = reinterpret_cast<int32_t*>(smem + Lo.ord);
  const bool grouped = (MODE != OPP) && R.task_group && R.n_groups > 1;
  const bool has_groups = (MODE != OPP) && R.task_group && R.group_anchor;
  const bool keyed = (MODE == CA_FF) && R.sort_hosts;

  if (CA)
    for (int i = tid; i < Z * Z; i += RES_THREADS) {
      const int a = i / Z, z = i - a * Z;
      csum[i] = R.cost[a * Z + z] + R.cost[z * Z + a];
      bsum[i] = R.bw[a * Z + z] + R.bw[z * Z + a];
    }
  for (int t = tid; t < T; t += RES_THREADS) R.placement[t] = -1;

  // hosts -> registers (padding slots never fit: -inf capacities)
  const int h0 = tid * HPL;
  double a0[HPL], a1[HPL], a2[HPL], a3[HPL], key[HPL], cc[HPL], bb[HPL];
  int32_t zz[HPL];
  uint32_t tb[HPL];
#pragma unroll
  for (int j = 0; j < HPL; j++) {
    const int h = h0 + j;
    const bool v = h < H;
    a0[j] = v ? R.avail[h] : -DINF;
    a1[j] = v ? R.avail[(size_t)H + h] : -DINF;
    a2[j] = v ? R.avail[2 * (size_t)H + h] : -DINF;
    a3[j] = v ? R.avail[3 * (size_t)H + h] : -DINF;
    zz[j] = (CA && v) ? R.zone[h] : 0;
    tb[j] = (MODE == VBP_BF && v) ? R.tiebreak[h] : 0u;
    key[j] = 0.0;                         // first-fit by index unless keyed
    cc[j] = 0.0;
    bb[j] = 1.0;
  }

  // a2: processing order (opportunistic keeps the caller's order)
  uint64_t* ka = reinterpret_cast<uint64_t*>(smem + Lo.u);
  uint64_t* kb = ka + A.Tpad;
  if (MODE == OPP) {
    for (int i = tid; i < T; i += RES_THREADS) ord[i] = i;
    __syncthreads();
  } else {
    res_order(R, grouped, R.sort_tasks != 0, ka, kb, ord, A.Tpad);
  }
  for (int i = tid; i < T; i += RES_THREADS) R.order[i] = ord[i];

  double* cd = reinterpret_cast<double*>(smem + Lo.cd);
  int32_t* c_anc = reinterpret_cast<int32_t*>(smem + Lo.ci);
  int32_t* c_caller = c_anc + RES_CHUNK;
  int32_t* c_grp = c_caller + RES_CHUNK;
  uint32_t* mk = reinterpret_cast<uint32_t*>(smem + Lo.mt) + wave * RES_MT_STRIDE;
  uint64_t* posts = reinterpret_cast<uint64_t*>(smem + Lo.slot);   // [2][WAVES][2]
  int32_t* cposts = reinterpret_cast<int32_t*>(posts);              // opp: [2][WAVES]
  MtWave mw;
  mw.buf = 0; mw.used = 0; mw.limit = 0;
  if (MODE == OPP) {
    const uint32_t* src = A.mt + (size_t)blockIdx.x * 625;
    for (int i = lane; i < 625; i += WAVE) mk[i] = src[i];
    __builtin_amdgcn_s_waitcnt(0xc07f);
  }

  int cur_anc = -1, cur_grp = -1;
  for (int p0 = 0; p0 < T; p0 += RES_CHUNK) {
    const int n = min(RES_CHUNK, T - p0);
    __syncthreads();                      // the previous chunk (and the sort keys) are consumed
    for (int i = tid; i < n; i += RES_THREADS) {
      const int t = ord[p0 + i];
      cd[i * 4 + 0] = R.dem[t];
      cd[i * 4 + 1] = R.dem[(size_t)T + t];
      cd[i * 4 + 2] = R.dem[2 * (size_t)T + t];
      cd[i * 4 + 3] = R.dem[3 * (size_t)T + t];
      const int g = has_groups ? R.task_group[t] : 0;
      c_anc[i] = has_groups ? R.group_anchor[g] : 0;
      c_caller[i] = t;
      c_grp[i] = g;
    }
    __syncthreads();
    for (int q = 0; q < n; q++) {
      const int p = p0 + q;
      const double d0 = cd[q * 4 + 0], d1 = cd[q * 4 + 1], d2 = cd[q * 4 + 2], d3 = cd[q * 4 + 3];
      const int t = c_caller[q];
      if (CA) {
        const int anc = c_anc[q];
        if (anc != cur_anc) {             // anchor rows of the zone tables -> registers
          cur_anc = anc;
#pragma unroll
          for (int j = 0; j < HPL; j++) { cc[j] = csum[anc * Z + zz[j]]; bb[j] = bsum[anc * Z + zz[j]]; }
        }
      }
      if (MODE == CA_FF && keyed) {
        const int g = c_grp[q];
        if (g != cur_grp) {               // frozen host key of the group (cost_aware.py:104-119)
          cur_grp = g;
#pragma unroll
          for (int j = 0; j < HPL; j++) {
            const double r = __builtin_sqrt(norm2_seq(a0[j], a1[j], a2[j], a3[j]));
            const double df = (R.decay && h0 + j < H) ? (double)R.decay[h0 + j] : 1.0;
            key[j] = (cc[j] * df) / (r * bb[j]);
          }
        }
      }
      const int par = p & 1;
      if (MODE == OPP) {
        // feasible hosts of this lane (np.all(r >= d), opportunistic.py:15)
        uint32_t fm = 0;
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < HPL; j++) {
          const bool f = fits<false>(a0[j], a1[j], a2[j], a3[j], d0, d1, d2, d3);
          fm |= (f ? 1u : 0u) << j;
          cnt += f ? 1 : 0;
        }
        const int inc = wave_incl_scan(cnt);
        const int wt = __builtin_amdgcn_readlane(inc, 63);
        if (lane == 0) cposts[par * RES_WAVES + wave] = wt;
        __syncthreads();
        int ntot = 0, off = 0;
#pragma unroll
        for (int w = 0; w < RES_WAVES; w++) {
          const int v = cposts[par * RES_WAVES + w];
          off += (w < wave) ? v : 0;
          ntot += v;
        }
        if (ntot == 0) continue;
        const int k = (int)mt_randint(mk, mw, (uint32_t)ntot) - off;   // randomizer.choice (:16)
        if (k >= 0 && k < wt && inc > k && inc - cnt <= k) {
          int rr = k - (inc - cnt);
#pragma unroll
          for (int j = 0; j < HPL; j++) {
            if ((fm >> j) & 1u) {
              if (rr == 0) {
                a0[j] -= d0; a1[j] -= d1; a2[j] -= d2; a3[j] -= d3;   // commit (:18)
                R.placement[t] = h0 + j;
              }
              rr--;
            }
          }
        }
        continue;
      }

      // lane best: (score bits, tiebreak:host), first minimum in host order
      uint64_t b1 = NONE, b2 = NONE;
#pragma unroll
      for (int j = 0; j < HPL; j++) {
        const bool f = fits<STRICT>(a0[j], a1[j], a2[j], a3[j], d0, d1, d2, d3);
        uint64_t k1 = 0;
        if (MODE == CA_BF || MODE == VBP_BF) {
          if (f) {
            const double s = __builtin_sqrt(norm2_seq(a0[j] - d0, a1[j] - d1, a2[j] - d2, a3[j] - d3));
            // cost_aware.py:83 (c * r * decay / bw, decay == 1); vbp.py:45 (la.norm)
            k1 = dbits(MODE == CA_BF ? (cc[j] * s) / bb[j] : s);
          }
        } else if (MODE == CA_FF) {
          k1 = dbits(key[j]);
        }
        const uint64_t k2 = ((uint64_t)tb[j] << 32) | (uint32_t)(h0 + j);
        if (f && (k1 < b1 || (k1 == b1 && k2 < b2))) { b1 = k1; b2 = k2; }
      }
      // wave minimum: score bits first; among tied lanes the first holds the lowest host
      // (blocked host mapping), except vbp best-fit, whose tiebreak rank precedes the host
      uint64_t m1 = b1;
#pragma unroll
      for (int off = 1; off < WAVE; off <<= 1) {
        const uint64_t o = shfl_xor_u64(m1, off);
        m1 = o < m1 ? o : m1;
      }
      const uint64_t tied = __ballot(b1 == m1);
      uint64_t m2 = readlane_u64(b2, __builtin_ctzll(tied));
      if (MODE == VBP_BF && __popcll(tied) > 1) {
        uint64_t c2 = (b1 == m1) ? b2 : NONE;
#pragma unroll
        for (int off = 1; off < WAVE; off <<= 1) {
          const uint64_t o = shfl_xor_u64(c2, off);
          c2 = o < c2 ? o : c2;
        }
        m2 = readlane_u64(c2, 0);
      }
      if (lane == 0) {
        posts[(par * RES_WAVES + wave) * 2 + 0] = m1;
        posts[(par * RES_WAVES + wave) * 2 + 1] = m2;
      }
      __syncthreads();
      uint64_t g1 = NONE, g2 = NONE;
#pragma unroll
      for (int w = 0; w < RES_WAVES; w++) {
        const uint64_t v1 = posts[(par * RES_WAVES + w) * 2 + 0];
        const uint64_t v2 = posts[(par * RES_WAVES + w) * 2 + 1];
        if (v1 < g1 || (v1 == g1 && v2 < g2)) { g1 = v1; g2 = v2; }
      }
      if (g2 == NONE) continue;          // no host fits: the task stays waiting
      const int hw = (int)(uint32_t)g2;
      if (hw / HPL == tid) {
        const int jw = hw - h0;
#pragma unroll
        for (int j = 0; j < HPL; j++)
          if (j == jw) { a0[j] -= d0; a1[j] -= d1; a2[j] -= d2; a3[j] -= d3; }   // resc[h] -= d
        R.placement[t] = hw;
      }
    }
  }

#pragma unroll
  for (int j = 0; j < HPL; j++) {
    const int h = h0 + j;
    if (h < H) {
      R.avail[h] = a0[j];
      R.avail[(size_t)H + h] = a1[j];
      R.avail[2 * (size_t)H + h] = a2[j];
      R.avail[3 * (size_t)H + h] = a3[j];
    }
  }
  if (MODE == OPP && wave == 0) {
    mt_unbuffer(mk, mw);
    uint32_t* dst = A.mt + (size_t)blockIdx.x * 625;
    for (int i = lane; i < 625; i += WAVE) dst[i] = mk[i];
  }
}

template <int MODE>
static void launch_mode(int hpl, int n, size_t lds, const ResidentArgs& a, hipStream_t st) {
  const dim3 grid(n), block(RES_THREADS);
  switch (hpl) {
    case 1: hipLaunchKernelGGL((resident_kernel<MODE, 1>), grid, block, lds, st, a); break;
    case 2: hipLaunchKernelGGL((resident_kernel<MODE, 2>), grid, block, lds, st, a); break;
    case 4: hipLaunchKernelGGL((resident_kernel<MODE, 4>), grid, block, lds, st, a); break;
    case 8: hipLaunchKernelGGL((resident_kernel<MODE, 8>), grid, block, lds, st, a); break;
    default: hipLaunchKernelGGL((resident_kernel<MODE, 16>), grid, block, lds, st, a); break;
  }
}

void launch_resident(int mode, int hpl, int n, const ResidentArgs& a, hipStream_t st) {
  const size_t lds = resident_lds_bytes(a.Zb, a.Tpad);
  switch (mode) {
    case CA_FF: launch_mode<CA_FF>(hpl, n, lds, a, st); break;
    case CA_BF: launch_mode<CA_BF>(hpl, n, lds, a, st); break;
    case OPP: launch_mode<OPP>(hpl, n, lds, a, st); break;
    case VBP_FF: launch_mode<VBP_FF>(hpl, n, lds, a, st); break;
    case VBP_BF: launch_mode<VBP_BF>(hpl, n, lds, a, st); break;
    default: break;
  }
}

template <int MODE>
static hipError_t attrs_mode(int lds) {
  hipError_t e = hipSuccess, r;
#define PVT_RES_ATTR(HPL)                                                                        \
  r = hipFuncSetAttribute((const void*)resident_kernel<MODE, HPL>,                               \
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds);                      \
  if (r != hipSuccess) e = r;
  PVT_RES_ATTR(1) PVT_RES_ATTR(2) PVT_RES_ATTR(4) PVT_RES_ATTR(8) PVT_RES_ATTR(16)
#undef PVT_RES_ATTR
  return e;
}

hipError_t resident_init_attrs() {
  const int lds = (int)resident_lds_bytes(ZMAX, RES_MAX_TASKS);
  hipError_t e = hipSuccess, r;
  if ((r = attrs_mode<CA_FF>(lds)) != hipSuccess) e = r;
  if ((r = attrs_mode<CA_BF>(lds)) != hipSuccess) e = r;
  if ((r = attrs_mode<OPP>(lds)) != hipSuccess) e = r;
  if ((r = attrs_mode<VBP_FF>(lds)) != hipSuccess) e = r;
  if ((r = attrs_mode<VBP_BF>(lds)) != hipSuccess) e = r;
  return e;
}

}  // namespace pvt
