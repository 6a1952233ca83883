// pvt_anchor.hip — mode-host anchor resolution (reference scheduler/cost_aware.py:45-58).
// See pvt_anchor.h for the rule. One wave per item: short lists counted in registers, longer
// ones sorted in the wave's LDS slice as (host + 1) << 32 | position keys (bitonic), every run
// end binary-searching its run start, and the wave keeps the max of (count << 32 | ~first).
// Lists beyond the wave's slice go to a block kernel (block-wide LDS sort, or LDS histograms
// over host ranges for lists longer than the block's tile).
// Integer-only, gather-bound: 4 B (8 B through inst_host) read per list entry.
#include "pvt_anchor_dev.h"

namespace pvt {

// The deferred long lists q = blk, blk + nblk, ... of one anchor call, one block each.
__device__ __forceinline__ void anchor_block_part(const AnchorArgs& a, int blk, int nblk) {
  __shared__ uint64_t lds[ANC_LDS];
  __shared__ uint64_t red[ANC_THREADS / 64];
  const int nd = *a.n_deferred;
  for (int q = blk; q < nd; q += nblk) {
    block_item(a, a.deferred[q], lds, red);
    __syncthreads();
  }
}

__global__ void __launch_bounds__(ANC_THREADS) anchor_block_kernel(AnchorArgs a) {
  anchor_block_part(a, blockIdx.x, gridDim.x);
}

__global__ void __launch_bounds__(ANC_THREADS) anchor_wave_kernel(AnchorArgs a) {
  __shared__ uint64_t lds[ANC_THREADS / 64][ANC_WLDS];
  const int wave = threadIdx.x >> 6;
  anchor_wave_item(a, blockIdx.x * (ANC_THREADS / 64) + wave, lds[wave]);
}

void launch_anchor(const AnchorArgs& a, hipStream_t st) {
  if (a.C <= 0) return;
  constexpr int IPB = ANC_THREADS / 64;
  anchor_wave_kernel<<<(a.C + IPB - 1) / IPB, ANC_THREADS, 0, st>>>(a);
  anchor_block_kernel<<<a.C < 256 ? a.C : 256, ANC_THREADS, 0, st>>>(a);
}

// Several anchor calls in one launch each (pvt_place_host_batch: the cost_aware rounds of a
// tick): block b of the wave launch serves call r with boff[r] <= b < boff[r + 1]; the block
// launch gives every call ANC_BATCH_BLOCKS blocks.
constexpr int ANC_BATCH_BLOCKS = 8;
__global__ void __launch_bounds__(ANC_THREADS) anchor_wave_batch_kernel(const AnchorArgs* A,
                                                                         const int32_t* boff, int nr) {
  __shared__ uint64_t lds[ANC_THREADS / 64][ANC_WLDS];
  int r = 0;
  while (r + 1 < nr && boff[r + 1] <= (int)blockIdx.x) r++;
  const AnchorArgs a = A[r];
  const int wave = threadIdx.x >> 6;
  anchor_wave_item(a, ((int)blockIdx.x - boff[r]) * (ANC_THREADS / 64) + wave, lds[wave]);
}
__global__ void __launch_bounds__(ANC_THREADS) anchor_block_batch_kernel(const AnchorArgs* A) {
  const AnchorArgs a = A[blockIdx.x / ANC_BATCH_BLOCKS];
  anchor_block_part(a, blockIdx.x % ANC_BATCH_BLOCKS, ANC_BATCH_BLOCKS);
}

int anchor_batch_blocks(int C) { constexpr int IPB = ANC_THREADS / 64; return (C + IPB - 1) / IPB; }

void launch_anchor_batch(const AnchorArgs* args_dev, const int32_t* boff_dev, int nr, int nblocks,
                         hipStream_t st) {
  if (nr <= 0) return;
  if (nblocks > 0) anchor_wave_batch_kernel<<<nblocks, ANC_THREADS, 0, st>>>(args_dev, boff_dev, nr);
  anchor_block_batch_kernel<<<nr * ANC_BATCH_BLOCKS, ANC_THREADS, 0, st>>>(args_dev);
}

}  // namespace pvt
