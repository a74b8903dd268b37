// ticket_wait.hpp -- the rare blocking wait of the persistent ticket sweeps (k_det_sweep2 in
// kernels_detsweep.hip, k_online_sweep in kernels_det.hip).  Included inside
// namespace mfhip { namespace { ... } }.
//
// The polling loop is one inline-asm block.  Written as a C++ loop (or as an out-of-line call), or
// left with an early return on failure, it made the compiler's wait counts of EVERY step of the
// sweep conservative -- the structurized exit / loop joins every later step, so each step waited
// for the rows loaded one step earlier instead of two: a memory round trip per update.  The
// callers therefore never return early: a wave that times out sets err and carries on, and every
// later wait then sees err at once (the host refuses the context when err is set).
#pragma once

// Poll *t until it equals want (returns 0), *err becomes non-zero (1) or ~2^20 polls pass (2,
// ~1-2 s: a producer never ran).  Agent-scope relaxed loads (sc1); ends with vmcnt(0), so every
// earlier memory operation of the wave has completed too.
__device__ __forceinline__ int poll_until(const int32_t* t, int32_t want, const int32_t* err) {
  int st, x;
  uint32_t n = 0;
  int32_t a, b;
  asm volatile(
      "1:\n\t"
      "global_load_dword %[a], %[z], %[t] sc1\n\t"
      "global_load_dword %[b], %[z], %[e] sc1\n\t"
      "s_waitcnt vmcnt(0)\n\t"
      "v_readfirstlane_b32 %[x], %[a]\n\t"
      "s_mov_b32 %[st], 0\n\t"
      "s_cmp_eq_u32 %[x], %[w]\n\t"
      "s_cbranch_scc1 2f\n\t"
      "v_readfirstlane_b32 %[x], %[b]\n\t"
      "s_mov_b32 %[st], 1\n\t"
      "s_cmp_lg_u32 %[x], 0\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_mov_b32 %[st], 2\n\t"
      "s_add_u32 %[n], %[n], 1\n\t"
      "s_cmp_gt_u32 %[n], %[lim]\n\t"
      "s_cbranch_scc1 2f\n\t"
      "s_sleep 1\n\t"
      "s_branch 1b\n\t"
      "2:"
      : [st] "=&s"(st), [x] "=&s"(x), [n] "+s"(n), [a] "=&v"(a), [b] "=&v"(b)
      : [t] "s"(t), [e] "s"(err), [z] "v"(0u), [w] "s"(want), [lim] "s"(1u << 20)
      : "scc", "memory");
  return st;
}

// A wave that timed out marks the launch failed (lane 0, agent scope) and carries on.
__device__ __forceinline__ void wait_ticket_or_fail(const int32_t* t, int32_t want, int32_t* err, int lane) {
  if (poll_until(t, want, err) == 2 && lane == 0)
    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
