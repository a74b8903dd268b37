// kernels.hpp -- host-side launch wrappers of the HIP kernels (kernels_det.hip, kernels_fast.hip,
// kernels_eval.hip).  All launches are asynchronous on the given stream.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "plan.hpp"

namespace mfhip {

// Update arithmetic of one replayed rating.
enum class Arith : int {
  kDsgd = 0,     // DSGDforMF.updateLocalFactors body (:405-413), regularised
  kSgdNext = 1,  // SGDUpdater.nextFactors (core/FactorUpdater.scala:37-45)
};

// Deterministic replay of one dependency level: one wave per entry, sequential dot.
// T = double (bit-exact) or float (fast-mode online).  eta = learning rate of the superstep
// (kDsgd) or SGDUpdater's learningRate (kSgdNext).
void launch_level(hipStream_t st, const DetEntry* entries, int64_t n, void* U, void* I,
                  const void* regU, const void* regI, int k, double eta, Arith arith, bool f64);
// Online micro-batch as one persistent launch (k_online_sweep, kernels_det.hip): wave w applies
// entries [wbeg[w], wbeg[w+1]) (the updates of its items, in sequence order), each after its
// user's ticket reaches useq; tickets (one int32 per user row) start at 0.  Every wave must be
// resident: nw <= online_sweep_capacity(k, f64).
int online_sweep_capacity(int k, bool f64);
void launch_online_sweep(hipStream_t st, int nw, const int64_t* wbeg, const DetEntry* ent, const uint32_t* useq,
                         void* U, void* I, int k, double eta, bool f64, int32_t* ticket, int32_t* err);
// The f32 batch at k <= 256 (k_online_f32, kernels_online_sweep.hip): the same plan and tickets,
// rows and tickets pipelined two updates deep, the dot product of online_f32.hpp (the f32 level
// replay's).  dummy_ticket: 16 int32 per wave of scratch.  skip (may be null): the launch does
// nothing when *skip != 0 (read on the device).  ev0 / ev1 (may be null) time the launch.
bool online_f32_supports(int k);
int online_f32_capacity(int k);
void launch_online_f32(hipStream_t st, int nw, const int64_t* wbeg, const DetEntry* ent, const uint32_t* useq, float* U,
                       float* I, uint64_t u_bytes, uint64_t i_bytes, int k, double eta, int32_t* ticket,
                       int32_t* dummy_ticket, int32_t* err, int nsingle, const int32_t* skip, hipEvent_t ev0,
                       hipEvent_t ev1);
// k_online_sweep's inputs from one batch in sequence order (eu / ei / er: user row, item row,
// rating of update x; device arrays), on the device (kernels_online.hip): ent / useq (n each,
// grouped by wave = item row mod W, sequence order inside a wave, useq = the update's rank among
// its user's updates) and wbeg (W + 1); touched[0..1] = distinct user / item rows of the batch.
// user_rows / item_rows bound eu / ei.  erf non-null: the ratings are floats there (the f32
// sweep's upload) and er is not read.
struct OnlineSweepScratch;
// Returns H: waves [0, H) hold one item each (the heavy items), the others any number.
uint32_t online_sweep_plan(hipStream_t st, OnlineSweepScratch& sc, const uint32_t* eu, const uint32_t* ei,
                           const double* er, int64_t n, uint32_t W, uint32_t user_rows, uint32_t item_rows,
                           DetEntry* ent, uint32_t* useq, int64_t* wbeg, int32_t* touched,
                           const float* erf = nullptr);
// The online batch's id -> row lookup on the device, over a mirror of the host IdIndex (same
// hash, same slots; id_index.hpp): in[0, n) user ids and in[n, 2n) item ids (the batch as
// uploaded) are replaced by their rows, 0xFFFFFFFF where the table has no such id; *misses counts
// those (the host then gives the unseen ids rows in first-touch order).  A null table: all misses.
void launch_id_lookup(hipStream_t st, uint32_t* in, int64_t n, const void* uslots, uint64_t umask, const void* islots,
                      uint64_t imask, int32_t* misses);
// slots[pos[j]] = vals[j] (8-B slots): the mirror takes the host table's writes since its last sync
void launch_id_scatter(hipStream_t st, void* slots, const uint32_t* pos, const void* vals, int64_t m);
// The f64 online batch on the deterministic sweep (kernels_detsweep.hip): the plan's entries as
// SoA arrays in sc.soa (eu / ei / eq / er, padded by kDetPad) and one DetWave per wave (single-item
// flag from the entries) into waves[0 .. W).  Call after online_sweep_plan on the same scratch.
void online_det_entries(hipStream_t st, OnlineSweepScratch& sc, const DetEntry* ent, const uint32_t* useq,
                        const int64_t* wbeg, int64_t n, uint32_t W, uint32_t*& eu, uint32_t*& ei, uint32_t*& eq,
                        double*& er, struct DetWave* waves);
// The deterministic sweep's superstep input built on the device (MFHIP_TEST det_build=host: on the
// host, plan.cpp build_det_step -- the same arrays, bit for bit).  One block of the superstep:
struct DetBuildBlock {
  int64_t e0;     // its first entry in the superstep's arrays
  int64_t st;     // its first rating in the device copy of RatingBlocks::det_aos
  int64_t iwoff;  // its item -> wave map in the concatenated maps
  uint32_t i0;    // first global item row of its item block
  uint32_t w0;    // its first wave in the superstep's wave order
};
static_assert(sizeof(DetBuildBlock) == 32, "DetBuildBlock is two 16-B words");
struct DetBuildScratch;
// ord[e0 + j] = the block's j-th rating in shuffle order (position inside the block, from the
// host's JVM shuffle); out = the entries in wave order (a wave's entries in shuffle order) with
// useq = the user's count of earlier ratings in shuffle order: exactly build_det_step's SoA.
// Reserve scratch for up to n_max entries first (det_device_build_reserve; no allocation after).
void det_device_build_reserve(DetBuildScratch& sc, int64_t n_max, uint32_t wave_bound, uint32_t user_rows);
void det_device_build(hipStream_t st, DetBuildScratch& sc, const int32_t* ord, int64_t n, const DetBuildBlock* blocks,
                      int nblk, const DetEntry* aos, const int32_t* item_wave, uint32_t wave_bound,
                      uint32_t user_rows, uint32_t* ou, uint32_t* oi, uint32_t* oq, double* orr);
// Per-rating records of the online operators (mf_online_update_out), f64 rows of k at
// [src[entry] * k]: kOutNext = (user', item') (FlinkOnlineMF.scala:131-135), kOutDelta =
// (user + deltaItem, deltaItem) with user before the update (PSOfflineOnlineMF.scala:174-176).
enum class OnlineOut : int { kNone = 0, kOutNext = 1, kOutDelta = 2 };
void launch_level_out(hipStream_t st, const DetEntry* entries, int64_t n, void* U, void* I, int k, double eta, bool f64,
                      OnlineOut mode, const int32_t* src, double* uout, double* iout);

// Fast-mode sweep, one rotation sub-step t for nblk rating blocks of one superstep.
struct FastBlk {
  int64_t rec_base;   // first record of the rating block
  int64_t cell_base;  // its G*G+1 cell offsets in the cell table
};
// Factor slabs are addressed through 32-bit buffer offsets (u_bytes/i_bytes < 4 GiB each).
// dummy_u_off / dummy_i_off: byte offsets of rows that are never written (idle prefetches of
// rows forwarded in registers).
// Cells of at least prio_len records run at raised wave priority (s_setprio 3).
void launch_fast_substep(hipStream_t st, const FastBlk* blks, int nblk, int G, int t, const FastRec* recs,
                         const int32_t* cell_off, float* U, float* I, int k, float eta, uint64_t u_bytes,
                         uint64_t i_bytes, uint32_t dummy_u_off, uint32_t dummy_i_off, int prio_len);

// Fast-mode sweep, one persistent launch per superstep: wave g of a block sweeps its G cells in
// order and waits on wave g+1's progress word before each cell (progress: nblk*G*kProgStride
// int32, zeroed before every launch; err[0] != 0 after a bounded wait timed out).
constexpr int kProgStride = 32;  // one 128-B line per progress word
void launch_fast_superstep(hipStream_t st, const FastBlk* blks, int nblk, int G, const FastRec* recs,
                           const int32_t* cell_off, float* U, float* I, int k, float eta, uint64_t u_bytes,
                           uint64_t i_bytes, uint32_t dummy_u_off, uint32_t dummy_i_off, int32_t* progress,
                           int32_t* err);

// Fast-mode sweep, pair schedule (kernels_pair.hip): one launch per sub-step, one wave per
// cell, two updates of one item per step (build_pair_plan).  k in {64, 128, 256}; the plan
// window must be >= 2 * pair_ring(pair_kpl(k)) (plan.hpp pair_window).
bool pair_kernel_supports(int k);
// ev0 / ev1 (may be null): start / stop events recorded by the dispatch itself.
void launch_sweep_pair(hipStream_t st, const WaveDesc* waves, int nwaves, const PairRec* recs, float* U, float* I,
                       uint64_t u_bytes, uint64_t i_bytes, int k, float eta, uint64_t* trace, hipEvent_t ev0,
                       hipEvent_t ev1);
// Systolic variant, one launch per superstep: sw = this superstep's PairPlan::sys_waves (nw of
// them, all of which must be resident at once: nw <= sweep_pair_sys_capacity(k)), sys =
// PairPlan::sys.  prog: nw*kProgStride int32 progress words, monotonic across launches (this
// launch writes base+1 .. base+G_j and must advance base by more than the largest G_j);
// err[0] is set when a wave gave up waiting.  trace (may be null): per cell {start, end} at
// [2*(cell index in sys)].
int sweep_pair_sys_capacity(int k);
// Hot-item replicas around a fast superstep (plan.hpp SplitItem): fork before the sweep, join
// after it, on the sweep's stream; n split items, f32 rows of k.
void launch_split_fork(hipStream_t st, const SplitItem* sp, int n, float* I, int k);
void launch_split_join(hipStream_t st, const SplitItem* sp, int n, float* I, int k);
// lbase: index of sw[0] among the superstep's waves (a superstep may be split over two launches,
// see mfhip.cpp ring overlap); prog and SysWave::nbr count from the superstep's first wave.
// place (may be null): block b of the launch sweeps wave sw[place[b]] (sys_placement, mfhip.cpp);
// null: the XCD-contiguous map.
void launch_sweep_pair_sys(hipStream_t st, const SysWave* sw, const WaveDesc* sys, int nw, int lbase,
                           const PairRec* recs, float* U, float* I, uint64_t u_bytes, uint64_t i_bytes, int k, float eta,
                           int32_t* prog, uint32_t base, int32_t* err, uint64_t* trace, hipEvent_t ev0, hipEvent_t ev1,
                           const int32_t* place = nullptr);

// Deterministic persistent sweep (kernels_detsweep.hip): one launch per superstep, nw waves of
// 64 lanes, all of which must be resident at once (nw <= det_sweep_capacity(k)).  Entries are
// build_det_step's SoA arrays; ticket: one int32 per user row, zero before the launch; err[0]
// set when a wave gave up waiting.  ev0 / ev1 (may be null): dispatch-recorded timing events.
int det_sweep_capacity(int k);
// Entry arrays are read in 64-entry chunks up to 192 entries past a wave's end (kDetPad slack).
// u_bytes / i_bytes: slab sizes (< 4 GiB, 32-bit row offsets); dummy_ticket: 16 scratch words
// per wave (nw * 16 int32).
constexpr int64_t kDetPad = 256;
void launch_det_sweep(hipStream_t st, const DetWave* waves, int nw, const uint32_t* eu, const uint32_t* ei,
                      const uint32_t* eq, const double* er, double* U, double* I, uint64_t u_bytes, uint64_t i_bytes,
                      const double* regU, const double* regI, int k, double eta, int32_t* ticket,
                      int32_t* dummy_ticket, int32_t* err, hipEvent_t ev0, hipEvent_t ev1);

// Split single-item chains (k = 64, 128, 256; kernels_detsweep.hip k_det_sweep_split): blocks of
// two wave slots, slots[2b + w] for wave w (nslots even, nslots / 2 blocks, all resident at once:
// nslots <= det_split_capacity(k), counted in wave slots; 0 = k not supported).  A block whose
// slot 0 is a single-item wave runs it as a chain wave plus a helper wave (slot 1 ignored, by
// convention kDetWaveHelper); any other slot is an ordinary k_det_sweep2 wave (count 0: none).
int det_split_capacity(int k);
// The same split sweep with SGDUpdater.nextFactors' update (the online f64 batch, no lambda /
// omega); k = 64, 128, 256 (capacity 0 otherwise).
int online_det_capacity(int k);
void launch_online_det(hipStream_t st, const DetWave* slots, int nslots, const uint32_t* eu, const uint32_t* ei,
                       const uint32_t* eq, const double* er, double* U, double* I, uint64_t u_bytes, uint64_t i_bytes,
                       int k, double eta, int32_t* ticket, int32_t* err, hipEvent_t ev0, hipEvent_t ev1);
void launch_det_sweep_split(hipStream_t st, const DetWave* slots, int nslots, const uint32_t* eu, const uint32_t* ei,
                            const uint32_t* eq, const double* er, double* U, double* I, uint64_t u_bytes,
                            uint64_t i_bytes, const double* regU, const double* regI, int k, double eta,
                            int32_t* ticket, int32_t* err, hipEvent_t ev0, hipEvent_t ev1);

// Gather-dot over resolved pairs (row -1 = unknown id).  out[j] = p.q summed left to right in
// f64 (predictRating's ddot).  When r != nullptr every workgroup writes partials[3*wg + c]:
//   c=0: sum (r - p.q)^2, c=1: matched count, c=2: sum mult*((r-p.q)^2 + lambda*(p.p + q.q)).
// The grid has predict_grid(n) workgroups; the host adds the partials in a fixed order.
int predict_grid(int64_t n);
void launch_predict(hipStream_t st, const int32_t* urow, const int32_t* irow, int64_t n,
                    const void* U, const void* I, int k, bool f64, double* out, const double* r,
                    const int32_t* mult, double lambda, double* partials);

// DSGD blocking on the device (kernels_block.hip): both SideLayouts (initFactorBlockAndIndices,
// DSGDforMF.scala:513-588, the reference's seeded blocking) and the rating blocks of user blocks
// [ub_lo, ub_hi) (:301-327; sort_ui: (user, item) order inside a block), bitwise what
// build_side + build_rating_blocks (plan.cpp) produce.  Host arrays in, host structures out.
class DevBuf;
// keep (optional): the rating blocks' device arrays (urow u32, irow u32, r f64, rb order, the
// first rb.start[n*n] entries valid) are handed over instead of freed.
struct DevRatingBlocks;
// host_arrays = false (with keep): rb gets only its block starts; fetch_rating_blocks copies the
// arrays later if a host-side plan needs them.
void device_blocking(hipStream_t st, const int32_t* u, const int32_t* i, const double* r, int64_t n, int32_t nb,
                     int64_t seed, int32_t ub_lo, int32_t ub_hi, bool sort_ui, SideLayout& U, SideLayout& I,
                     RatingBlocks& rb, DevRatingBlocks* keep = nullptr, bool host_arrays = true);
void fetch_rating_blocks(hipStream_t st, const DevRatingBlocks& dr, RatingBlocks& rb);
// Per rating block (n*n): the rating count of its most rated item, from the device arrays.
std::vector<int64_t> device_block_tops(hipStream_t st, const DevRatingBlocks& dr, const RatingBlocks& rb,
                                       const SideLayout& I);

// The fast pair schedule's per-cell work on the device (kernels_plan.hip): the greedy emission of
// every cell of `work` (build_fast_plan's phase-1 output, blocks in ascending order) and the pair
// records of every wave, bitwise the host build_fast_plan + build_pair_plan.  Fills fp's cell /
// record offsets and pads, pp's tables and stats (pp.recs stays empty) and d_pairs (device).
void device_pair_schedule(hipStream_t st, std::vector<FastBlockWork>& work, FastPlan& fp, int32_t nb, int32_t c,
                          int32_t shard, int32_t k, uint32_t dummy_row, int32_t window, bool substep_waves,
                          PairPlan& pp, DevBuf& d_pairs);
// The whole fast schedule from the device rating blocks (kernels_plan.hip): phase 1 as device
// sorts (cell-major order, spreading) around host LPT groups from device histograms, then the
// emission and pair records as above.  Gb: the rotation groups of every rating block.
void device_fast_schedule(hipStream_t st, const DevRatingBlocks& dr, const RatingBlocks& rb, const SideLayout& U,
                          const SideLayout& I, const std::vector<int32_t>& Gb, double lambda, uint64_t order_seed,
                          FastPlan& fp, int32_t c, int32_t shard, int32_t k, uint32_t dummy_row, int32_t window,
                          PairPlan& pp, DevBuf& d_pairs);

// Initial factor rows on the device (DSGDforMF.scala:548-549, MatrixFactorization.scala:278-280):
// row x, factor f = the f-th nextDouble of new Random(ids[x] ^ seed) (xor_seed) or of
// new Random(ids[x]).  One thread per element: the JVM LCG state after m steps is
// jump[2(m-1)] * s0 + jump[2(m-1)+1] mod 2^48 (host table, m = 1..2k), so every element is
// computed independently and written coalesced; bit-exact with JavaRandom::nextDouble.
// out: rows x k, double (f64) or float (rounded from the same double).
void launch_jvm_init_rows(hipStream_t st, const int32_t* ids, int64_t rows, int k, bool xor_seed, int64_t seed,
                          const uint64_t* jump, void* out, bool f64);

}  // namespace mfhip
