// plan.hpp -- host-side DSGD blocking and the two device schedules.
//
//  * SideLayout       initFactorBlockAndIndices (DSGDforMF.scala:513-588)
//  * RatingBlocks     rating-block construction (DSGDforMF.scala:301-327, toRatingBlockId :597-601)
//  * DetStratum       deterministic mode: one superstep's rating blocks in the reference's
//                     shuffled order (:392-393), grouped into dependency levels so that a level
//                     holds no two updates sharing a user or item row (bitwise == sequential)
//  * FastBlock        fast mode: each rating block split into G item groups x G user groups;
//                     sub-step t pairs item group g with user group (g+t) mod G, so every
//                     in-flight update owns its user and item row (conflict-free batching)
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "id_index.hpp"

namespace mfhip {

// Allocator whose resize() leaves trivially constructible elements uninitialised: the multi-GB
// record tables are filled by parallel writers, which then also take the first-touch page faults
// (a value-initialising resize zeroes them on one thread first).
template <class T>
struct NoInitAlloc : std::allocator<T> {
  template <class U> struct rebind { using other = NoInitAlloc<U>; };
  NoInitAlloc() = default;
  template <class U> NoInitAlloc(const NoInitAlloc<U>&) noexcept {}
  template <class U> void construct(U* p) noexcept { ::new (static_cast<void*>(p)) U; }
  template <class U, class... A> void construct(U* p, A&&... a) { ::new (static_cast<void*>(p)) U(std::forward<A>(a)...); }
};
template <class T>
using RecVec = std::vector<T, NoInitAlloc<T>>;

// Asks for transparent huge pages on a large, not yet touched buffer (first-touch faults then come
// 2 MB at a time instead of 4 KB: seconds on the multi-GB record tables).  Only a hint.
void hugepage_hint(void* p, size_t bytes);
template <class V>
void resize_huge(V& v, size_t n) {
  v.resize(n);
  hugepage_hint(v.data(), n * sizeof(typename V::value_type));
}

struct SideLayout {
  int32_t n_blocks = 1;
  std::vector<int32_t> row_id;       // row -> id; rows grouped by block, ids ascending in a block
  std::vector<int32_t> omega;        // row -> number of ratings of the id (:537-541)
  std::vector<int32_t> row_block;    // row -> factor block
  std::vector<int64_t> block_start;  // n_blocks + 1
  IdIndex index;                     // id -> row
  int64_t rows() const { return static_cast<int64_t>(row_id.size()); }
};

// How ids are assigned to factor blocks.
//  kJvm:      the reference's new Random(id ^ seed).nextInt(n) (DSGDforMF.scala:531-533).  Its
//             first draw varies slowly with the id, so runs of ~1.4k consecutive ids share a
//             block and rating blocks come out unequal (NFLX, n=8: largest 1.8x the mean).
//  kBalanced: fast-mode option: heaviest ids first into the least-loaded block (LPT over
//             rating counts, ties by a hash of id ^ seed), so all n*n rating blocks are near
//             equal and a superstep is not held up by one oversized block.  It changes which
//             ratings share a stratum, and with it the trajectory: on the NFLX-shaped synthetic
//             the held-out RMSE after 10 epochs is 0.690 against the reference blocking's 0.759.
enum class Blocking { kJvm, kBalanced };

// Builds the factor-block layout of one side from the rating column `ids`.
// has_seed: block = new Random(id ^ seed).nextInt(n) and ids sorted in a block;
// otherwise blocks come from an unseeded generator (the reference's scala.util.Random).
void build_side(SideLayout& s, const int32_t* ids, int64_t n, int32_t n_blocks, int64_t seed,
                bool has_seed, Blocking blocking = Blocking::kJvm);

// Per-rating global rows (parallel lookup).
void lookup_rows(const SideLayout& s, const int32_t* ids, int64_t n, std::vector<uint32_t>& rows);

struct RatingBlocks {
  int32_t n_blocks = 1;
  std::vector<int64_t> start;   // n*n + 1, block b = ub*n + ib
  RecVec<uint32_t> urow;        // global user row
  RecVec<uint32_t> irow;        // global item row
  RecVec<double> r;
  std::vector<int64_t> src;     // input index per position (only when requested)
  // deterministic sweep only: (urow, irow, r) interleaved, 16 B per rating, so the host build's
  // shuffle-order gather reads one cache line per rating instead of three (prepare_det_sweep)
  std::vector<struct DetEntry> det_aos;
  int64_t size(int64_t b) const { return start[b + 1] - start[b]; }
};

// Rating blocks for user blocks [ub_lo, ub_hi).  sort_ui reproduces the (user, item) order
// the reference imposes when seeded (:319-323; ties keep input order).
void build_rating_blocks(RatingBlocks& rb, const SideLayout& U, const SideLayout& I,
                         const int32_t* u, const int32_t* i, const double* r, int64_t n,
                         int32_t ub_lo, int32_t ub_hi, bool sort_ui, bool keep_src = false);

// ---------------------------------------------------------------------------------------
// Deterministic mode.
struct DetEntry {
  uint32_t u;  // global user row
  uint32_t i;  // global item row
  double r;
};

struct LevelPlan {
  std::vector<DetEntry> entries;      // level-major
  std::vector<int64_t> level_start;   // levels + 1
  int64_t levels() const { return static_cast<int64_t>(level_start.size()) - 1; }
};

// Appends a sequence (in its exact sequential order) to per-row last-level trackers and
// returns per-entry levels; rows of distinct sequences must be disjoint.
// Groups a set of independent ordered sequences into one level plan.
struct OrderedSeq {
  const uint32_t* u;
  const uint32_t* i;
  const double* r;
  const int32_t* order;  // may be null (identity)
  int64_t len;
  uint32_t u_lo, u_hi, i_lo, i_hi;  // row ranges touched (for the level trackers)
};
// src (optional): per entry, its index e into the sequence's u / i / r arrays (single sequence).
void build_level_plan(const std::vector<OrderedSeq>& seqs, LevelPlan& out, std::vector<int32_t>* src = nullptr);

// Deterministic mode, one persistent launch per superstep (kernels_detsweep.hip).  Every item
// of a rating block belongs to one wave (LPT over rating counts, fixed for the whole fit), which
// applies the updates of its items in the reference's shuffled order (DSGDforMF.scala:392-413);
// the only cross-wave dependency left is a user's previous update, which the wave awaits through
// a per-user ticket (useq = the number of earlier updates of that user in the superstep).  Every
// wave's entries are in increasing shuffle position, so the unfinished entry with the smallest
// position can always run: with all waves resident the sweep cannot deadlock.
constexpr uint32_t kDetUseqMask = (1u << 30) - 1;
// (round 4 also carried "same item as the previous / next entry" bits here, found by a host pass over
// every entry; the sweep now compares the entries' items itself)
struct DetWave {
  int64_t begin;  // first entry
  int32_t count;
  int32_t flags;  // kDetWaveSingleItem
};
constexpr int32_t kDetWaveSingleItem = 1;  // every entry of the wave updates one item
constexpr int32_t kDetWaveHelper = 2;      // split sweep: the helper slot of a single-item wave
static_assert(sizeof(DetWave) == 16, "DetWave is one 16-B word");

struct DetSweepLayout {
  std::vector<int32_t> block_waves;             // n*n: waves of each rating block of this shard (0: none)
  std::vector<std::vector<int32_t>> item_wave;  // n*n: local item row of the block's item block -> wave
  std::vector<std::vector<uint8_t>> wave_single;  // n*n: per wave of the block, 1 = it holds one item
};
// waves_per_superstep: budget of resident waves for one superstep of this shard; every block of a
// superstep gets a share proportional to its ratings (>= 1, <= its distinct items).
void build_det_layout(DetSweepLayout& L, const RatingBlocks& rb, const SideLayout& U, const SideLayout& I, int32_t c,
                      int32_t shard, int32_t waves_per_superstep);

// Host scratch of build_det_step, kept by the caller across supersteps (per staging slot), so
// the ~24 B per rating it gathers into are not page-faulted in again every superstep.
struct DetStepScratch {
  std::vector<RecVec<int32_t>> order, wv;
  std::vector<RecVec<uint32_t>> gu, gi;
  std::vector<RecVec<double>> gr;
};

// One superstep's entries (SoA, wave-major, each wave in shuffle-position order) for the rating
// blocks `blocks` with their shuffle seeds (order = scala_shuffle(new Random(seed)), :392-393;
// seeded = false: a random seed).  Sizes: waves = sum of block_waves, entries = sum of block sizes.
struct DetStepOut {
  DetWave* waves;
  uint32_t* u;   // global user row
  uint32_t* i;   // global item row
  uint32_t* qf;  // useq
  double* r;
};
int64_t det_build_phase_ns(int phase);  // MFHIP_TIMING diagnostics of build_det_step (0..4)
void build_det_step(const RatingBlocks& rb, const SideLayout& U, const SideLayout& I, const DetSweepLayout& L,
                    const std::vector<int64_t>& blocks, const std::vector<int64_t>& seeds, bool seeded,
                    const DetStepOut& out,
                    DetStepScratch* scratch = nullptr);

// ---------------------------------------------------------------------------------------
// Fast mode.
// Fast-mode record (32 B).  The kernel reads the first five words: byte offsets of the user
// and item rows in their slabs (row * k * 4) and the three per-update scalars.  Inside a cell
// no user occurs twice within kHazardWindow consecutive records (the kernel prefetches user
// rows that far ahead); where reordering inside an item run cannot achieve that, the plan
// inserts padding records: user = the zeroed dummy row, r = ru = ri = 0, item = the run's item.
// Such a record is an exact no-op of the update arithmetic (e = 0, the item row scaled by 1),
// so the kernel needs no flag; kPadBit in `i` marks it for host-side tools and tests.
constexpr uint32_t kPadBit = 0x80000000u;
constexpr int kHazardWindow = 8;
struct FastRec {
  uint32_t u_off;  // user row byte offset in the user slab
  uint32_t i_off;  // item row byte offset in the item slab
  float r;
  float ru;        // lambda / omega_u (f32)
  float ri;        // lambda / omega_i (f32)
  uint32_t u;      // global user row (the dummy row for padding)
  uint32_t i;      // global item row (| kPadBit for padding)
  uint32_t pad_;
};
static_assert(sizeof(FastRec) == 32, "FastRec is two 16-B words");

// Hot-item replicas (fast mode, opt-in `split_run`): inside one rating block an item with m >
// split_run ratings is swept as R = ceil(m / split_run) independent chains -- replica 0 is the
// item's own row, replicas 1..R-1 are scratch rows -- and averaged when the superstep ends:
//   fork:  scratch[0 .. R-2] = q
//   join:  q = (q + sum_{r=1..R-1} q_r) / R
// (iterative parameter mixing; a delta sum q0 + sum_r (q_r - q0) diverges: each chain of
// thousands of updates converges on its own, and R such corrections overshoot R-fold).
// Every in-flight update still owns the physical rows it touches (no atomics), but the item's
// updates are no longer one sequential chain: a relaxation of DSGDforMF.scala:404-413 that
// shortens the hottest item's chain by R (fast mode is judged on held-out RMSE, not order).
struct SplitItem {
  uint32_t main_row;     // the item's global row
  uint32_t scratch_row;  // first of R-1 scratch rows: replicas 1..R-1
  int32_t R;
};

// One rating of a block while its fast plan is built: index in the block, local user, local
// (virtual) item, rating.
struct PlanEnt { uint32_t x, ul, vil; float r; };

// A block after phase 1 of build_fast_plan (LPT groups, cell-major order, spreading): its
// entries in final cell order, ready for the greedy emission (host, or kernels_plan.hip).
struct FastBlockWork {
  int64_t b = 0;                       // rating block
  int64_t len = 0, nu = 0, nv = 0, ub = 0, GG = 0, T = 0;
  std::vector<int64_t> cstart;         // GG + 1 cell starts in e
  RecVec<PlanEnt> e;                   // the block's ratings in cell order
  std::vector<uint32_t> vrow;          // virtual item -> physical row
  std::vector<float> regu, regi;       // lambda / omega (f32) per local user / virtual item
};

struct FastPlan {
  int32_t G = 4;                       // rotation groups per rating block (the largest when per-block)
  std::vector<int32_t> Gb;             // per rating block (n*n): its rotation groups
  RecVec<FastRec> recs;                // all rating blocks of this shard, cell-major per block
  std::vector<int64_t> rec_base;       // per rating block (n*n), -1 if not on this shard
  std::vector<int32_t> cell_off;       // per included rating block: Gb*Gb+1 relative offsets
  std::vector<int64_t> cell_base;      // per rating block: index into cell_off (-1 if absent)
  int64_t pads = 0;                    // padding records inserted
  std::vector<SplitItem> splits;       // hot-item replicas, grouped by rating block
  std::vector<int64_t> split_off;      // n*n + 1: rating block b owns splits [split_off[b], split_off[b+1])
  std::shared_ptr<void> scratch;       // the builder's per-block working arrays (the caller may free them late)
  uint32_t scratch_rows = 0;           // scratch item rows used from scratch_base on
};

// ---------------------------------------------------------------------------------------
// Per-cell sweep launch table (kernels_pair.hip): one wave per cell.
constexpr uint32_t kOffOOB = 0xFFFFF000u;  // a row byte offset past any slab: load 0 / no store
struct WaveDesc {
  int64_t base;   // first record
  int32_t steps;  // records
  int32_t cells;
};

// ---------------------------------------------------------------------------------------
// Fast mode, pair schedule (kernels_pair.hip): a step applies two consecutive updates A, B of
// one cell with distinct users -- of the same item ("run" pair) or of two items ("split"
// pair, A ends its item run, B starts one); a step whose B would repeat A's user gets a
// no-op B.  Row fields are byte offsets, kOffOOB = no load (the row is forwarded in registers
// or the record is a no-op) / no store.
// The plan's hazard window (pair_window(k) >= 2 * pair_ring(KPL) records): a user row is loaded
// pair_ring pairs before its update, so inside a cell a user recurs either at the next record
// (forwarded in registers) or at least that far on; kPairPlanRing bounds the ring.  The sweeps prefetch pair_ring(KPL) <= kPairPlanRing pairs
// ahead (8 VMEM operations per pair, vmcnt <= 63), measured per row width (round 5,
// profiles/r05_pair_ring.txt): a deeper ring is NOT faster -- the pair step is not load-latency
// bound, and fewer rows in flight per wave leave the CU's memory path less crowded and a cell's
// ring prefill shorter: NFLX (KPL 2) 21.0 -> 20.27 ms at 6, ML20M (KPL 1) 4.93 -> 4.82 at 4,
// YAHOO (KPL 4) 237 -> 230 ms at 4.  Records come in chunks of pair_chunk(KPL) pairs (one per lane,
// a multiple of the ring).  Single-run waves (kWaveSingleRun, 4 VMEM ops per pair) use the same
// ring; build_pair_plan checks that every user row such a wave loads was last stored at least
// pair_ring pairs earlier (or is forwarded in registers).
constexpr int kPairPlanRing = 7;
#ifdef MFHIP_EXP_PAIR_RING  // experiment: one ring depth / chunk for every row width
constexpr int pair_ring(int) { return MFHIP_EXP_PAIR_RING; }
constexpr int pair_chunk(int) { return MFHIP_EXP_PAIR_CHUNK; }
#else
constexpr int pair_ring(int kpl) { return kpl == 2 ? 6 : 4; }
constexpr int pair_chunk(int kpl) { return kpl == 2 ? 60 : 56; }
#endif
// The window argument of build_fast_plan / device_fast_schedule: the low 16 bits are the hazard
// window of cells with several item runs, the high 16 bits (0: the same) that of single-item
// cells (one item run, the hot items' chains).  A run window also forbids a user at the next record
// (no forwarded repeats): the single-run block step (kernels_pair.hip) solves whole blocks of
// records at once and prefetches their rows two blocks ahead, so inside a cell no user may recur
// within run-window records.
constexpr int32_t plan_window_pack(int32_t w, int32_t run_w) { return (w & 0xFFFF) | (run_w << 16); }
constexpr int32_t plan_window_mixed(int32_t p) { return p & 0xFFFF; }
constexpr int32_t plan_window_run(int32_t p) { return (p >> 16) ? (p >> 16) : (p & 0xFFFF); }
constexpr bool plan_window_strict_runs(int32_t p) { return (p >> 16) != 0; }
constexpr int pair_kpl(int k) { return k <= 64 ? 1 : k <= 128 ? 2 : 4; }
// The plan window for k (>= 2 * pair_ring; MFHIP_TEST pair_window=N overrides it): 10 records at
// k = 64 (ML20M 4.82 / 4.49 / 4.45 / 4.64 ms at 14 / 8 / 10 / 12), 2 * kPairPlanRing = 14 above (NFLX
// 20.8 / 20.05 / 20.25 / 20.5 ms at 12 / 14 / 16 / 18, YAHOO 232 vs 215 ms at 8 vs 14; a wider window
// pads more, a narrower one orders the cells worse; profiles/r05_pair_ring.txt)
constexpr int pair_window(int k) { return k <= 64 ? 10 : 2 * kPairPlanRing; }
// The single-item cells' window for k (plan_window_pack; 0 = pair_window with forwarded repeats)
constexpr int pair_run_window(int) { return 0; }
static_assert(pair_window(64) >= 2 * pair_ring(pair_kpl(64)) && pair_window(128) >= 2 * pair_ring(pair_kpl(128)) &&
                  pair_window(256) >= 2 * pair_ring(pair_kpl(256)),
              "the hazard window covers the ring at every supported k");
static_assert(pair_chunk(1) % pair_ring(1) == 0 && pair_chunk(2) % pair_ring(2) == 0 &&
                  pair_chunk(4) % pair_ring(4) == 0, "ring slots must repeat every chunk");
static_assert(pair_ring(1) <= kPairPlanRing && pair_ring(2) <= kPairPlanRing && pair_ring(4) <= kPairPlanRing &&
                  pair_chunk(1) <= 64 && pair_chunk(2) <= 64 && pair_chunk(4) <= 64,
              "the plan window covers the ring; a chunk is one record per lane");
// Flags are one byte each (0 or 1), so the kernel turns each into a float coefficient with a
// single v_cvt_f32_ubyteN.
constexpr uint32_t kPairFwdA = 1u << 0;    // A's user row = previous pair's A result (registers)
constexpr uint32_t kPairFwdB = 1u << 8;    // A's user row = previous pair's B result
constexpr uint32_t kPairKeepQ = 1u << 16;  // A continues the item row held in registers
constexpr uint32_t kPairSplit = 1u << 24;  // B's item differs from A's (B starts a run)
constexpr int32_t kWaveGeneric = 1;    // WaveDesc.cells: generic pair steps
constexpr int32_t kWaveSingleRun = 2;  // the cell is one item run with no forwarded user row: no item traffic per pair
constexpr int32_t kWaveSingleRunFwd = 3;  // one item run, some A rows forwarded from the previous pair
struct PairRec {
  uint32_t ua, ub, ia, ib;   // loads: users A and B; items of A (run start) and B (split)
  uint32_t sa, sb, sia, si;  // stores: users A and B; A's item (split), the item after B (run end)
  uint32_t flags;
  float ra, rb, rua, rub, ria, rib;  // ratings and lambda/omega (0 for no-op records)
  uint32_t pad_;  // keeps the record four 16-B words
};
static_assert(sizeof(PairRec) == 64, "PairRec is four 16-B words");
// Systolic sweep wave: its G cells are PairPlan::sys[cell0 .. cell0+G), one per sub-step; it
// waits on wave nbr (same superstep) -- item group g+1 of the same rating block.
struct SysWave {
  int64_t cell0;
  int32_t G;
  int32_t nbr;
};
static_assert(sizeof(SysWave) == 16, "SysWave is one 16-B word");

struct PairPlan {
  RecVec<PairRec> recs;
  std::vector<int64_t> wave_cell;  // per wave: its cell, indexed like FastPlan::cell_off (cell_base[b] + cell)
  std::vector<int64_t> wave_sys;   // per wave: its slot in sys (-1: none)
  std::vector<WaveDesc> waves;   // one per non-empty cell (steps = pairs), every (sm, t), sm-major
  std::vector<int64_t> sub_off;  // nb*G + 1
  // Systolic tables (k_sweep_pair_sys): the waves of superstep sm are
  // sys_waves[sys_off[sm] .. sys_off[sm+1]) (local block j major, then item group g); their
  // cells live in sys (steps = 0 for an empty cell).
  std::vector<WaveDesc> sys;
  std::vector<SysWave> sys_waves;
  std::vector<int64_t> sys_off;
  std::vector<int64_t> sys_block_off;  // nb * (c+1): first wave of local block j in superstep sm, relative to sys_off[sm]
  int64_t noop_halves = 0;       // pair halves that are no-ops (planner padding, repeated users)
  std::vector<double> sm_bytes;  // per superstep index: bytes the sweep requests (records + in-range rows)
};
// The plan window must be >= 2 * pair_ring(pair_kpl(k)) records (pair_window(k) is; the knob
// MFHIP_TEST pair_window=N is clamped to it, mfhip.cpp plan_window).  substep_waves: order the cells (and
// pp.waves / sub_off) per sub-step (sm, t), longest first, for the per-sub-step launches (needs a
// uniform G); otherwise per superstep, and only the systolic tables are meaningful.
// cell_pairs (tables only): the pair count of every cell, indexed like fp.cell_off; the records
// are then built elsewhere (kernels_plan.hip) and pp.recs stays empty, pp.waves[].cells generic.
void build_pair_plan(PairPlan& pp, const FastPlan& fp, int32_t nb, int32_t c, int32_t shard, int32_t k,
                     bool substep_waves = true, const std::vector<int32_t>* cell_pairs = nullptr);

int32_t choose_groups(int64_t avg_block_ratings, int32_t blocks_per_device, int32_t fast_waves,
                      double cell_target = 150.0, int32_t default_waves = 2048);

// rec_src (optional): for every record, its position in the RatingBlocks arrays (-1: padding).
// dummy_row: user row used by padding records (kept zero by the caller).  k: row length in
// floats (record offsets are row * k * 4 and must stay below 4 GiB).
// window: a row recurs inside a cell only at the next position or >= window positions later
// (the kernel's prefetch distance; kHazardWindow for kernels_fast.hip).
// block_groups (optional, n*n): per rating block rotation groups (0 = G); otherwise G for all.
// split_run > 0: hot-item replicas (SplitItem) with scratch item rows from scratch_base on.
void build_fast_plan(FastPlan& fp, const RatingBlocks& rb, const SideLayout& U, const SideLayout& I,
                     int32_t G, int32_t k, double lambda, uint64_t order_seed, uint32_t dummy_row,
                     std::vector<int64_t>* rec_src = nullptr, int32_t window = kHazardWindow,
                     const std::vector<int32_t>* block_groups = nullptr, int32_t split_run = 0,
                     uint32_t scratch_base = 0, std::vector<FastBlockWork>* entries_out = nullptr);

// Longest-processing-time assignment of rows (by load) to G groups, as build_fast_plan's phase 1
// does for the users and items of a rating block (kernels_plan.hip uses it on device counts).
void lpt_assign(const std::vector<int64_t>& load, int32_t G, std::vector<int32_t>& group);

// Rotation groups per rating block for the systolic sweep, where every rating block of a
// superstep is its own G_j x G_j grid and only the superstep's longest wave matters.  For each
// superstep of this shard it picks the smallest G_j (multiples of 8) that bring every block's
// longest wave under a common bound T, with T minimal such that sum_j G_j <= waves.  A wave's
// time is modelled as G cells x kSysCellNs + max(block ratings / G, ratings of the block's
// most rated item) / 2 pairs x ns per pair (no group is lighter than one item's run).
constexpr double kSysCellNs = 6000.0;     // per-cell start, drain, hand-off and waiting (swept on NFLX + ML20M)
// With the round-5 rings the cell cost re-swept lower at k <= 128 (profiles/r05_group_model.txt:
// ML20M 4.65 -> 4.49 ms, NFLX 20.03 -> 19.97 ms at 5 us); k = 256 keeps 6 us (its 5-us schedule moves
// YAHOO@0.05's RMSE past the 0.5% gate).
// Round 6, with the record preload at k = 64 (profiles/r06_ML20M_cell_ab.txt): k = 64 re-swept to
// 3.5 us per cell and 230 ns per run pair (ML20M 4.26 -> 4.13 ms); NFLX keeps 186 ns (210 / 230 /
// 170 / 155 ns: 20.45 / 21.17 / 20.23 / 21.20 ms against 19.87) and, with the CU isolation, 4.5 us
// per cell (19.47 / 19.43 ms against 19.73 / 19.45 at 5 us; 5.5 / 4 us: 19.77 / 19.76, 19.76 / 19.71).
constexpr double sys_cell_ns(int k) { return k <= 64 ? 3500.0 : k <= 128 ? 4500.0 : kSysCellNs; }
constexpr double kSysPairNs = 300.0;      // mixed-cell pair step incl. no-op halves and group imbalance (tuned)
constexpr double kSysRunPairNs = 186.0;   // single-item-run pair step (wave trace)
constexpr double sys_run_pair_ns(int k) { return k <= 64 ? 230.0 : kSysRunPairNs; }
// split_run > 0: an item's run counts at most split_run ratings (hot-item replicas).
std::vector<int32_t> choose_block_groups(const RatingBlocks& rb, const SideLayout& I, int32_t c, int32_t shard,
                                         int32_t waves, int32_t split_run = 0, double cell_ns = kSysCellNs,
                                         double run_ns = kSysRunPairNs);
// The same model on per-block rating counts and most-rated-item counts (size / top, n*n each,
// shard blocks only; e.g. from device histograms, kernels_plan.hip device_block_tops).
std::vector<int32_t> choose_block_groups(const std::vector<int64_t>& size, const std::vector<int64_t>& top, int32_t nb,
                                         int32_t c, int32_t shard, int32_t waves, double cell_ns = kSysCellNs,
                                         double run_ns = kSysRunPairNs);

}  // namespace mfhip
