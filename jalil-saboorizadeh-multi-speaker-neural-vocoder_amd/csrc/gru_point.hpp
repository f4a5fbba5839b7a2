// Pointwise GRU backward shared by the per-step kernel (gru.hip) and the persistent sweep
// (gru_seq.hip).  Contraction is off so both round identically (and like an unfused fp32
// reference): given dh and the forward's r, z, n, gh_n, h_{t-1}
//   dn = dh (1-z)   dz = dh (h_{t-1} - n)   da_n = dn (1 - n^2)
//   da_r = da_n gh_n r (1-r)   da_z = dz z (1-z)   dgh_n = da_n r   dh_direct = dh z
#pragma once

struct GruBwdPoint {
    float dar, daz, dghn, dan, ddir;
};

__device__ __forceinline__ GruBwdPoint gru_bwd_point(float dh, float r, float z, float n,
                                                     float ghn, float hp) {
#pragma clang fp contract(off)
    GruBwdPoint o;
    const float dn = dh * (1.0f - z);
    const float dz = dh * (hp - n);
    o.dan = dn * (1.0f - n * n);
    const float dr = o.dan * ghn;
    o.dar = dr * r * (1.0f - r);
    o.daz = dz * z * (1.0f - z);
    o.dghn = o.dan * r;
    o.ddir = dh * z;
    return o;
}
