// Device body of plik_lite's deferred quadratic form fed by raw window sums
// (the sampler's split pipelined steps: steptail.hip's step tail and
// sampler.hip's unified step launch).
#pragma once

#include "divrn.h"
#include "qftile.h"
#include "steptail.h"

namespace cmamd {

typedef double f64x4 __attribute__((ext_vector_type(4)));

// Quadratic-form workgroup LDS (doubles): the A operand's two BK buffers,
// reused after the K loop by the epilogue's Delta_I tile (64 x 66); then the
// tile's cal^2 per walker, the item's X over its K range and over its I panel.
static constexpr int QFS_TILE_D = QF_TILE * (QF_TILE + 2);
static_assert(QFS_TILE_D >= 2 * QF_TILE * BK, "the Delta_I tile reuses the operand buffers");
static constexpr int QFS_LDS_DOUBLES = QFS_TILE_D + QF_TILE + QF_MAXKB * QF_TILE + QF_TILE;

// plik_lite's deferred quadratic form (quadform_body<false>, quadform.hip)
// with its B operand formed in registers instead of LDS-DMA'd: lane (li, lk)
// of wave v multiplies walker 16 v + li's k = 8 lk .. 8 lk + 7 of every BK
// step, so it loads exactly those raw sums itself (a step ahead, beside the
// A tile's LDS-DMA) and forms Delta = X - S / cal^2 with the window pass's
// emit operations (theorypass_body.h): the fragments, the MFMA order and the
// epilogue are quadform_body's, so the partials are the same bits as the
// deferred launch over the pass's Delta rows.  The A panel (C^-1) is still
// shared through LDS; without B there the workgroup needs 37 KB instead of
// 64, so it fits beside the window pass's workgroups.
// SIGNAL (the unified step launch, sampler.hip): the partials are stored
// agent-scope (write-through) for a consumer in the same launch.
template <bool SIGNAL = false>
__device__ __forceinline__ void qfs_body(double *smem, int item_ix, int tile, const QFSArgs &a)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const QFSource &q = a.src;
    const int Np = q.Np, W = a.W;
    const int w0 = tile * QF_TILE;
    const QFItem it = q.items[item_ix];
    const int nsteps = it.nJ * (QF_TILE / BK);
    const int kbase0 = it.J0 * QF_TILE;
    const double *Arow = q.Ct + (size_t)(it.I * QF_TILE) * Np;
    double *c2s = smem + QFS_TILE_D;            // [64] cal^2 of the tile's walkers
    double *xs = c2s + QF_TILE;                 // [nJ * 64] X over the item's K range
    double *xI = xs + QF_MAXKB * QF_TILE;       // [64] X over the I panel
    dma_tile(smem, Arow, Np, kbase0, wave, lane);
    const double *Srow = a.S + (size_t)(w0 + 16 * wave + li) * Np + kbase0 + 8 * lk;
    double2 sv[4];
#pragma unroll
    for (int u = 0; u < 4; u++) sv[u] = *reinterpret_cast<const double2 *>(Srow + 2 * u);
    if (tid < QF_TILE) {                        // the emit's c2 = cal * cal (walkers past W: never stored)
        const int wc = min(w0 + tid, W - 1);
        double cl = 1.0;
        if (a.cal_index >= 0) cl = a.nuis[(long long)wc * a.ld_nuis + a.cal_index];
        c2s[tid] = cl * cl;
        xI[tid] = q.X[it.I * QF_TILE + tid];
    }
    for (int i = tid; i < it.nJ * QF_TILE; i += 256) xs[i] = q.X[kbase0 + i];
    f64x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; t++) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    double c2 = 1.0, rc2 = 1.0;
    for (int s = 0; s < nsteps; s++) {
        const int buf = s & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();                        // A tile s and this lane's sums landed; buf^1 free
        if (s == 0) {
            c2 = c2s[16 * wave + li];
            rc2 = 1.0 / c2;
        }
        double2 b[4];
        {
            const double *xk = xs + s * BK + 8 * lk;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const double2 x2 = *reinterpret_cast<const double2 *>(xk + 2 * u);
                b[u].x = x2.x - div_rn(sv[u].x, c2, rc2);
                b[u].y = x2.y - div_rn(sv[u].y, c2, rc2);
            }
        }
        if (s + 1 < nsteps) {
            dma_tile(smem + (buf ^ 1) * QF_TILE * BK, Arow, Np, kbase0 + (s + 1) * BK, wave, lane);
#pragma unroll
            for (int u = 0; u < 4; u++) sv[u] = *reinterpret_cast<const double2 *>(Srow + (s + 1) * BK + 2 * u);
        }
        const double *A = smem + buf * QF_TILE * BK;
        double2 af[4][4];
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int r = 16 * t + li;
#pragma unroll
            for (int u = 0; u < 4; u++)
                af[t][u] = *reinterpret_cast<const double2 *>(A + r * BK + (((lk * 4 + u) ^ swz(r)) * 2));
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
#pragma unroll
            for (int t = 0; t < 4; t++)
                acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[t][u].x, b[u].x, acc[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 4; t++)
                acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[t][u].y, b[u].y, acc[t], 0, 0, 0);
        }
    }
    // Delta_I tile: smem[n][i] (row stride QF_TILE + 2), as quadform_body
    double2 dI[QF_TILE * QF_TILE / 2 / 256];
#pragma unroll
    for (int u = 0; u < QF_TILE * QF_TILE / 2 / 256; u++) {
        const int e = tid + 256 * u, r = e >> 5, c = (e & 31) * 2;
        dI[u] = *reinterpret_cast<const double2 *>(a.S + (size_t)(w0 + r) * Np + it.I * QF_TILE + c);
    }
    __syncthreads();                            // every wave done with the operand buffers
#pragma unroll
    for (int u = 0; u < QF_TILE * QF_TILE / 2 / 256; u++) {
        const int e = tid + 256 * u, r = e >> 5, c = (e & 31) * 2;
        double2 v = make_double2(0.0, 0.0);
        if (w0 + r < W) {
            const double cr = c2s[r], rr = 1.0 / cr;
            v.x = xI[c] - div_rn(dI[u].x, cr, rr);
            v.y = xI[c + 1] - div_rn(dI[u].y, cr, rr);
        }
        *reinterpret_cast<double2 *>(smem + r * (QF_TILE + 2) + c) = v;
    }
    __syncthreads();
    const int n = 16 * wave + li;
    double sacc = 0.0;
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) sacc += acc[t][r] * smem[n * (QF_TILE + 2) + 16 * t + lk + 4 * r];
    sacc += __shfl_xor(sacc, 16);
    sacc += __shfl_xor(sacc, 32);
    if (lk == 0) {
        double *p = q.partial + ((size_t)tile * q.n_items + item_ix) * QF_TILE + n;
        if (SIGNAL)
            __hip_atomic_store(p, sacc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        else
            *p = sacc;
    }
}

}  // namespace cmamd
