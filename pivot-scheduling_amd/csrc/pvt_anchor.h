// pvt_anchor.h — anchor resolution for cost_aware groups.
//
// The reference groups each ready task by the storage of the zone of its predecessors' MODE
// host (scheduler/cost_aware.py:45-58):
//     preds = [t for p in app.get_predecessors(c.id) for t in p.tasks]
//     placement, _ = max(Counter([t.placement for t in preds]).items(), key=lambda x: x[1])
// Counter keeps first-insertion order and max() returns the first maximum, so the mode is the
// host with the highest count and, among equal counts, the earliest first occurrence in the
// predecessor list. On the GPU: one wave per item (a container of ready tasks). Up to 64
// entries are counted in registers; up to ANC_WLDS are sorted in the wave's LDS slice as
// 64-bit keys (host + 1) << 32 | position, each run end finding its run start by binary search,
// and the wave keeps the max of (count, ~first position). Longer lists are deferred to a block
// kernel: a block-wide LDS sort up to ANC_LDS entries, beyond that passes over host ranges of
// ANC_LDS hosts (between the list's min and max host) building LDS histograms of (count, first
// position). No global scratch, so items may share rows of a resident list table.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pvt {

constexpr int ANC_THREADS = 256;
constexpr int ANC_WLDS = 1024;   // keys a wave sorts alone (8 KiB of LDS per wave)
constexpr int ANC_LDS = 8192;    // block kernel: 64 KiB of LDS per workgroup; longer are counted

struct AnchorArgs {
  int C, H;
  int64_t n_pred, n_inst, n_rows;
  const int64_t* off;       // [C+1], or [n_rows+1] when item is set
  const int32_t* item;      // optional [C]: the row of off for each item
  const int32_t* list;      // [n_pred] host index (or instance index when inst_host is set)
  const int32_t* inst_host; // optional [n_inst]: host per instance, -1 = not placed
  const int32_t* zone;      // [H]
  int32_t* mode_host;       // [C] out
  int32_t* anchor_zone;     // [C] out
  int32_t* bad;             // [1] count of items with an invalid range or host index
  int32_t* deferred;        // [C] items whose lists exceed ANC_WLDS (block kernel)
  int32_t* n_deferred;      // [1]
};

void launch_anchor(const AnchorArgs& a, hipStream_t st);
// nr anchor calls (their AnchorArgs in device memory) in two launches: the wave launch has
// nblocks = the sum of anchor_batch_blocks(C) blocks, call r starting at boff[r]
int anchor_batch_blocks(int C);
void launch_anchor_batch(const AnchorArgs* args_dev, const int32_t* boff_dev, int nr, int nblocks,
                         hipStream_t st);

}  // namespace pvt
