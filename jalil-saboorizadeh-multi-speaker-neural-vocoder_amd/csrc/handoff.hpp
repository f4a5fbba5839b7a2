// In-launch hand-offs between workgroups of a persistent kernel (gen_mlp.hip, gru_xcd.hip).
//
// Data-tagged granules (MI355X guide, Guideline 16 R2): an 8-byte {value, tag} word written
// by ONE store and polled with L1-bypassing (sc1) loads -- the data is its own flag, so no
// fence, flag or barrier sits between producer and consumer.  Global mode stores write
// through (sc1) so any XCD sees them; local mode (all members of a group proved to run on
// this XCD by hx_group_local) uses plain stores that stay in the XCD's shared L2.
#pragma once
#include "common.hpp"

typedef unsigned long long u64;

namespace hx {
constexpr int SPIN_LIMIT = 1 << 20;    // polls (each >= one L2 round trip): ~ a second
// error words (the per-call word and the sticky flag, persist.hip, keep the largest)
constexpr int ERR_HANDOFF = 1;         // a hand-off never arrived within the spin limit
constexpr int ERR_RESIDENCY = 2;       // the group's workgroups were not all resident in time
// the arrival wait is bounded by wall time, not by the hand-off spin count: 30 s of
// s_memrealtime (100 MHz).  Work of other kernels holding CUs when a sweep starts only delays
// its late workgroups (they start when those kernels end), so it must not be an error.
constexpr unsigned long long ARRIVAL_TICKS = 3000000000ull;
}

__device__ __forceinline__ void hx_put(u64* p, uint32_t tag, uint32_t v, bool local) {
    const u64 x = ((u64)tag << 32) | v;
    if (local)
        __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    else
        __hip_atomic_store(p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Buffer resource over a hand-off buffer: 16-B granule-pair loads with sc1 (L1 bypass)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t hx_rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff,
                                             0x00020000);
}
__device__ __forceinline__ uint4 hx_get2(__amdgpu_buffer_rsrc_t r, uint32_t byte_off) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16 /*sc1*/);
    uint4 u;
    __builtin_memcpy(&u, &v, 16);
    return u;
}

// One poll of a bounded spin: sleeps, and returns true (give up) once the spin limit is hit
// (raising the error word) or another workgroup raised it.
__device__ __forceinline__ bool hx_spin_fail(int& spins, int* err, int lane, int sleep = 1,
                                             int limit = hx::SPIN_LIMIT) {
    for (int i = 0; i < sleep; ++i) __builtin_amdgcn_s_sleep(1);
    if (++spins > limit) {
        if (lane == 0)
            __hip_atomic_fetch_max(err, hx::ERR_HANDOFF, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        return true;
    }
    if ((spins & 31) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        return true;
    return false;
}

// words of one placement-check array ([G][P] slots, G * P <= HX_KEYED_WORDS)
#define HX_KEYED_WORDS 520

// Co-residency.  Every member of a group waits for every other member's hand-offs, so a
// group is only safe once ALL its members are resident.  The host guarantees that the grid
// fits the device (srnn_persist_fits: occupancy x CUs >= workgroups x processes sharing the
// device) -- so every workgroup does start, at the latest when the kernels that held CUs at
// launch time have ended -- and each member first waits for the whole group to arrive
// (hx_group_local below) with no spin bound, only a 30-s wall-time guard.  The hand-off spin
// limit then only counts polls among resident workgroups.
//
// Group placement check.  The static map (group g = block % G, member p = block / G) puts a
// whole group on one XCD when blocks are dealt round-robin over the 8 XCDs and G % 8 == 0;
// the hand-offs can then stay in that XCD's L2 (local mode).  Every member writes
// 1 + its XCC id to its slot of a zeroed [G][P] array (agent scope: visible across XCDs),
// and one wave per member reads the group's P slots until all are written: the group is
// local iff they all name the same XCC.  All members read the same final slots, so they
// all take the same decision; placement only changes speed, never correctness.  One
// store and one read round trip per member, all in parallel (a shared arrival counter
// would serialise its atomics across the grid).
__device__ __forceinline__ unsigned hx_xcc_id() {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    return xcc & 7;
}
__device__ __forceinline__ void hx_group_arrive(int* slot) {
    __hip_atomic_store(slot, 1 + (int)hx_xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// whole wave; slots = the group's P words.  Waits until every member has arrived (the
// co-residency gate above; ERR_RESIDENCY after ARRIVAL_TICKS), then returns whether they all
// run on one XCD (and allow_local).
__device__ __forceinline__ bool hx_group_local(int* slots, int P, int* err, int allow_local = 1) {
    const int lane = threadIdx.x & 63;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool same = true;
    for (int q0 = 0; q0 < P; q0 += 64) {
        const int q = min(q0 + lane, P - 1);
        int v = 0, polls = 0;
        for (;;) {
            v = __hip_atomic_load(slots + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__ballot(v == 0) == 0) break;
            __builtin_amdgcn_s_sleep(2);
            if ((++polls & 63) == 0) {
                if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                    return false;
                if (__builtin_amdgcn_s_memrealtime() - t0 > hx::ARRIVAL_TICKS) {
                    if (lane == 0)
                        __hip_atomic_fetch_max(err, hx::ERR_RESIDENCY, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
                    return false;
                }
            }
        }
        const int v0 = __builtin_amdgcn_readfirstlane(v);
        same = same && __ballot(v != v0) == 0 &&
               (q0 == 0 || v0 == __hip_atomic_load(slots, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT));
    }
    return same && allow_local;
}
