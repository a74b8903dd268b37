/*
 * mfhip_testing.h -- test hooks of libmfhip.so.  NOT part of the product surface (mfhip.h):
 * the test suite and tools/ use these to check the device schedules' invariants on a CPU
 * machine and to name the kernels in profiles.  The Scala/JNI drop-in never binds them.
 */
#ifndef MFHIP_TESTING_H
#define MFHIP_TESTING_H

#include "mfhip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Testing hooks (host only, no GPU): expose the device schedules so their invariants can be
   checked on a CPU machine.
   mf_debug_levels: dependency level of each update of a sequence visited in `order`
   (order may be NULL = identity); rows are caller indices.
   mf_debug_fast_schedule: for every input rating, the rating block (ub*n+ib), rotation
   sub-step, item group and position inside its cell of the fast-mode plan with `groups`
   groups per rating block (groups < 0: the systolic sweep's per-block choice for a budget of
   -groups waves per superstep, as mf_dsgd_prepare makes it with MFHIP_TEST=sys_waves=-groups for
   rank k: the group model's constants depend on the row width, plan.hpp sys_cell_ns /
   sys_run_pair_ns), MF_BLOCKING_* `blocking` and hazard window `window` (0: 8). */
int mf_debug_levels(const uint32_t* urow, const uint32_t* irow, const int32_t* order, int64_t n,
                    int32_t* level_out);
int mf_debug_fast_schedule(const int32_t* users, const int32_t* items, int64_t n, int32_t n_blocks,
                           int64_t seed, int32_t groups, int32_t blocking, int32_t window, int32_t k,
                           int32_t* block_out, int32_t* substep_out, int32_t* group_out, int64_t* pos_out);
/* mf_debug_fast_split: mf_debug_fast_schedule with hot-item replicas (the MFHIP_ITEM_SPLIT
   experiment, item_split ratings per chain); replica_out[j] = 0 when rating j updates its item's own row, r >= 1 when it
   updates replica r (merged when the superstep ends). */
int mf_debug_fast_split(const int32_t* users, const int32_t* items, int64_t n, int32_t n_blocks,
                        int64_t seed, int32_t groups, int32_t blocking, int32_t window, int32_t k, int32_t item_split,
                        int32_t* block_out, int32_t* substep_out, int32_t* group_out, int64_t* pos_out,
                        int32_t* replica_out);
/* mf_debug_ring_schedule: the item-block ring step ring_shift runs after superstep `superstep`
   (1-based) on rank `rank` of `world` with n blocks (n = c * world): the item block it sends
   (*out_blk) to rank *dst and the one it receives (*in_blk) from rank *src -- nextRatingBlock
   (DSGDforMF.scala:611-619) over ranks. */
int mf_debug_ring_schedule(int32_t rank, int32_t world, int32_t n_blocks, int64_t superstep, int32_t* out_blk,
                           int32_t* in_blk, int32_t* dst, int32_t* src);
/* mf_debug_plan_digest: after mf_dsgd_prepare of a fast-mode fit on one shard, an FNV-1a digest
   of the device schedule -- the pair records, the wave table and (systolic) the per-wave cell
   tables -- and the pair-record count: out[0] = digest, out[1] = records.  Compares the device-
   built plan (kernels_plan.hip) with the host-built one (MFHIP_TEST=device_plan=0). */
int mf_debug_plan_digest(mf_ctx* ctx, uint64_t out[2]);
/* The plan window (records between two uses of a row inside a cell unless adjacent) the fast
   sweep uses at rank k: the prefetch distance of the kernel selected for k. */
int mf_fast_plan_window(int32_t k, int32_t* window_out);
/* Name of the fast-mode sweep kernel used at rank k (for profiles and bench reports). */
const char* mf_fast_kernel_name(int32_t k);
/* Build flags: bit 0 = built with -DMFHIP_EXPERIMENTS (hot-item replicas, wave traces and the
   other experiment switches exist; the default build has none of them). */
int32_t mf_debug_build_flags(void);
/* Device memory this process holds through the library: out[0] = live bytes, out[1] = the
   high-water mark since the library was loaded (rank rehearsals report it per rank). */
int mf_debug_device_bytes(int64_t out[2]);

#ifdef __cplusplus
}
#endif
#endif /* MFHIP_TESTING_H */
