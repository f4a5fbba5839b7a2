// In-launch hand-offs between workgroups of a persistent kernel (gen_mlp.hip, gru_xcd.hip).
//
// Data-tagged granules (MI355X guide, Guideline 16 R2): an 8-byte {value, tag} word written
// by ONE store and polled with L1-bypassing (sc1) loads -- the data is its own flag, so no
// fence, flag or barrier sits between producer and consumer.  Global mode stores write
// through (sc1) so any XCD sees them; local mode (all members of a group proved to run on
// this XCD by hx_census) uses plain stores that stay in the XCD's shared L2.
#pragma once
#include "common.hpp"

typedef unsigned long long u64;

namespace hx {
constexpr int SPIN_LIMIT = 1 << 20;    // polls (each >= one L2 round trip): ~ a second
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
        if (lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return true;
    }
    if ((spins & 31) == 0 && __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
        return true;
    return false;
}

// XCD census (one lane per workgroup).  cur: 9 zeroed words ([0..8) per-XCC slot counters,
// [8] arrivals).  Every workgroup takes a slot on its XCD (s_getreg XCC_ID) and waits for all
// arrivals; if every XCD holds whole groups of P members, groups are formed per XCD
// (g = groups on lower XCDs + slot / P, p = slot % P) and true is returned (local mode).
// Otherwise g, p keep the caller's static map.  All workgroups read the same final counts,
// so they all take the same decision.  Placement only changes speed, never correctness.
__device__ __forceinline__ bool hx_census(int* cur, int P, int* err, int& g, int& p) {
    unsigned xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    xcc &= 7;
    const int slot = __hip_atomic_fetch_add(cur + xcc, 1, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    // (the arrival depends on the slot, so it issues after the count is performed; relaxed:
    //  an agent-scope release / acquire would write back / invalidate the whole L2)
    __hip_atomic_fetch_add(cur + 8, 1 + (slot >> 30), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int spins = 0;
    while (__hip_atomic_load(cur + 8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
           (int)(gridDim.x * gridDim.y)) {
        if (hx_spin_fail(spins, err, 0)) return false;
    }
    int ok = 1, before = 0;
    for (int x = 0; x < 8; ++x) {
        const int c = __hip_atomic_load(cur + x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok &= c % P == 0;
        if (x < (int)xcc) before += c;
    }
    if (!ok) return false;
    g = before / P + slot / P;
    p = slot % P;
    return true;
}

// Keyed census: the member index p of every workgroup is fixed by the caller (so everything
// that depends only on p -- resident weight fragments -- can be loaded before the census);
// only the group g is assigned.  cur: HX_KEYED_WORDS zeroed words ([x * 64 + p] per-XCC
// per-member counters, [512] arrivals), P <= 64.  Local mode iff on every XCD all P members
// occur equally often: then the c_x groups of XCD x take indices [sum_{x'<x} c_x', + c_x)
// and the member's slot picks one.  Otherwise g keeps the caller's static value.
#define HX_KEYED_WORDS 520
// Split in two so the caller can issue its own loads between arrival and the wait.
// Returns this member's slot on its XCD.
__device__ __forceinline__ int hx_census_arrive(int* cur, int p, unsigned& xcc) {
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    xcc &= 7;
    const int slot = __hip_atomic_fetch_add(cur + xcc * 64 + p, 1, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
    // (data-dependent on the slot, so ordered after the count without a release fence,
    //  which at agent scope would write back the whole L2)
    __hip_atomic_fetch_add(cur + 512, 1 + (slot >> 30), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return slot;
}
// Called by a whole wave (uniform slot / xcc, from the arriving lane): lane q reads the
// 8 per-XCC counters of member q at once, so the check costs one round trip, not 8 x P.
__device__ __forceinline__ bool hx_census_finish(int* cur, int P, int slot, unsigned xcc,
                                                 int* err, int& g) {
    const int lane = threadIdx.x & 63;
    int spins = 0;
    while (__hip_atomic_load(cur + 512, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
           (int)(gridDim.x * gridDim.y)) {
        if (hx_spin_fail(spins, err, lane)) return false;
    }
    const int q = min(lane, P - 1);
    int v[8];
#pragma unroll
    for (int x = 0; x < 8; ++x)
        v[x] = __hip_atomic_load(cur + x * 64 + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool ok = true;
    int before = 0;
#pragma unroll
    for (int x = 0; x < 8; ++x) {
        const int c = __shfl(v[x], 0);
        ok = ok && __ballot(v[x] != c) == 0;
        before += x < (int)xcc ? c : 0;
    }
    if (!ok) return false;
    g = before + slot;
    return true;
}
