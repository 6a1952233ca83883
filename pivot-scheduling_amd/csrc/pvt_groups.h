// pvt_groups.h — cost_aware grouping on the device (pvt_groups.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace pvt {

constexpr int GRP_MAX_TASKS = 16384;   // tasks of a fused round (keys in registers, 16 per thread)
constexpr int GRP_MAX_KEYS = 8192;     // storages + applications (LDS table)

struct CaGroupArgs {
  int T, C, Z, S, n_apps;
  const int32_t* task_item;     // [T]
  const int32_t* anchor_zone;   // [C] from the anchor kernels: zone, -1 none, -2 unplaced, -3 bad
  const int32_t* item_app;      // [C]
  const int32_t* storage_zone;  // [S]
  const int32_t* zone_storage;  // [Z]
  uint32_t* mt;                 // [625] the policy's MT19937 state, in/out
  int32_t* task_group;          // [T] out
  int32_t* group_anchor;        // [>= groups] out
  int32_t* status;              // [2] out: groups, error kind
  int32_t* desc_n_groups;       // the device round descriptor's n_groups, or NULL
};
void launch_ca_groups(const CaGroupArgs& a, hipStream_t st);
void launch_ca_groups_batch(const CaGroupArgs* args_dev, int n, hipStream_t st);

}  // namespace pvt
