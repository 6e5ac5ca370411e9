// Device body of plik_lite's deferred quadratic form fed by raw window sums
// (sampler.hip's unified step launch).
#pragma once

#include "divrn.h"
#include "qftile.h"
#include "steptail.h"

namespace cmamd {

typedef double f64x4 __attribute__((ext_vector_type(4)));

// Quadratic-form workgroup LDS (doubles): three BK buffers of the A operand
// (the K loop's two, and a third so that its last step leaves two free for the
// epilogue's raw Delta_I rows); then the item's X over its K range and over
// its I panel.
static constexpr int QFS_NBUF = 3;
static constexpr int QFS_BUF_D = QF_TILE * BK;
static constexpr int QFS_XS_D = 3 * 128;         // the K range's X: three waves' 1 KB DMA pieces
static_assert(QFS_XS_D >= QF_MAXKB * QF_TILE, "X over an item's K range");
static constexpr int QFS_LDS_DOUBLES = QFS_NBUF * QFS_BUF_D + QFS_XS_D + QF_TILE;

// One operand buffer's 16 KB by LDS-DMA, 16 pieces of 1 KB, 4 a wave: either
// the A tile at column k0 (dma_tile's layout), or 32 rows of the tile's raw
// sums over the I panel (S rows w0 + 32 h .. + 31, columns col0 .. col0 + 63;
// two rows a piece, the 16-byte chunk c of row r stored at chunk c ^ (r & 15)
// so the epilogue's reads of one column by 16 rows spread over the banks).
__device__ __forceinline__ void dma_next(double *buf, bool a_tile, const double *Arow, int k0, const double *Sw0,
                                         int col0, int h, size_t Np, int wave, int lane)
{
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int piece = wave * 4 + q;
        const int ra = piece * 4 + (lane >> 4);
        const int rs = 32 * h + 2 * piece + (lane >> 5);
        // (selected by mask: a uniform branch here splits the block, and the
        // compiler's wait counts turn pessimistic across the joins)
        const uintptr_t pa = (uintptr_t)(Arow + (size_t)ra * Np + k0 + ((lane & 15) ^ swz(ra)) * 2);
        const uintptr_t ps = (uintptr_t)(Sw0 + (size_t)rs * Np + col0 + ((lane & 31) ^ (rs & 15)) * 2);
        const uintptr_t m = (uintptr_t)0 - (uintptr_t)a_tile;
        const double *src = (const double *)((pa & m) | (ps & ~m));
        __builtin_amdgcn_global_load_lds((gbl_void_t *)src, (lds_void_t *)(buf + piece * 128), 16, 0, 0);
    }
}

typedef double f64x2 __attribute__((ext_vector_type(2)));

// A K step's LDS reads as asm blocks.  The compiler waits for every LDS-DMA in
// flight before any LDS read it emits itself (it cannot tell the buffers
// apart), which would make the two-step-ahead loads wait on the next step;
// these reads touch only buffers whose DMA the step's s_waitcnt has covered.
// qfs_a_reads<u>: the A fragments a[t] of rows 16 t + li, chunk lk * 4 + u
// (swz(16 t + li) = swz(li), so row t's chunk is row li's + 4 KB t; abase[u] is
// row li's LDS byte address); qfs_x_reads: the X values x[u] at k = 8 lk + 2 u.
template <int U>
__device__ __forceinline__ void qfs_a_reads(const unsigned (&abase)[4], f64x2 (&a)[4])
{
    asm volatile(
        "ds_read_b128 %0, %4 offset:0\n"
        "ds_read_b128 %1, %4 offset:4096\n"
        "ds_read_b128 %2, %4 offset:8192\n"
        "ds_read_b128 %3, %4 offset:12288\n"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(a[0]), "=&v"(a[1]), "=&v"(a[2]), "=&v"(a[3])
        : "v"(abase[U]));
}

__device__ __forceinline__ void qfs_x_reads(unsigned xbase, f64x2 (&x)[4])
{
    asm volatile(
        "ds_read_b128 %0, %4 offset:0\n"
        "ds_read_b128 %1, %4 offset:16\n"
        "ds_read_b128 %2, %4 offset:32\n"
        "ds_read_b128 %3, %4 offset:48\n"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(x[0]), "=&v"(x[1]), "=&v"(x[2]), "=&v"(x[3])
        : "v"(xbase));
}

__device__ __forceinline__ unsigned lds_addr(const double *p)
{
    return (unsigned)(size_t)((const __attribute__((address_space(3))) double *)p);
}

// Loads the compiler does not see (no wait of its own): the caller waits
// with a counted vmcnt and passes the registers through that asm.
__device__ __forceinline__ void qfs_load4(const double *p, f64x2 (&v)[4])
{
    asm volatile(
        "global_load_dwordx4 %0, %4, off\n"
        "global_load_dwordx4 %1, %4, off offset:16\n"
        "global_load_dwordx4 %2, %4, off offset:32\n"
        "global_load_dwordx4 %3, %4, off offset:48"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3])
        : "v"(p));
}

__device__ __forceinline__ double qfs_load1(const double *p)
{
    double v;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=&v"(v) : "v"(p));
    return v;
}

// plik_lite's deferred quadratic form (quadform_body<false>, quadform.hip)
// with its B operand formed in registers instead of LDS-DMA'd: lane (li, lk)
// of wave v multiplies walker 16 v + li's k = 8 lk .. 8 lk + 7 of every BK
// step, so it loads exactly those raw sums itself and forms
// Delta = X - S / cal^2 with the window pass's emit operations
// (theorypass_body.h): the fragments, the MFMA order and the epilogue's sums
// are quadform_body's, so the partials are the same bits as the deferred
// launch over the pass's Delta rows.  The A panel (C^-1) is shared through
// LDS, one K step ahead.  This form (items of one or two column blocks) DMAs
// the epilogue's Delta_I rows during the last K step instead of loading them
// after it, and each lane forms its own 16 Delta_I values as it sums: the
// accept-only launch that ends a step call, where the quadratic form is the
// critical path, 24.1-24.4 -> 21.3-21.8 us.  In the middle launches, beside
// the pass, it measured 0.2 us slower than qfs_body_loop (the chi^2 beside it
// slows), and distance-2 prefetch 0.7 us slower: qfs_body_loop runs there.
// SIGNAL (the unified step launch, sampler.hip): the partials are stored
// agent-scope (write-through) for a consumer in the same launch.
template <int NJ, bool SIGNAL>
__device__ __forceinline__ void qfs_body_nj(double *smem, int item_ix, int tile, const QFSArgs &a)
{
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    const QFSource &q = a.src;
    const int Np = q.Np, W = a.W;
    const int w0 = tile * QF_TILE;
    const QFItem it = q.items[item_ix];
    // unrolled: an asm load's registers are in flight into the next step, and a
    // loop's back edge may copy them (reading them before they land)
    constexpr int nsteps = NJ * (QF_TILE / BK);   // even, >= 2
    const int kbase0 = it.J0 * QF_TILE;
    const double *Arow = q.Ct + (size_t)(it.I * QF_TILE) * Np;
    double *xs = smem + QFS_NBUF * QFS_BUF_D;   // [nJ * 64] X over the item's K range
    double *xI = xs + QFS_XS_D;                 // [64] X over the I panel
    const double *Sw0 = a.S + (size_t)w0 * Np;
    const int n = 16 * wave + li;               // this lane's walker in the tile
    // The VGPR loads (the calibration, the raw sums) are inline asm waited for
    // by hand: beside LDS-DMA the compiler waits vmcnt(0) for any load of its
    // own (cdna_hip_programming.md, the LDS-DMA GEMM traps), which at the last
    // step would wait for the Delta_I rows too.  Every vector memory operation
    // counts in issue order; each step's own wait covers both queues.
    // tools/check_asm_loads.py (tests/test_codeobj.py) checks the built code.
    double cv;
    const bool has_cal = a.cal_index >= 0;
    {                                           // the emit's c2 = cal * cal (walkers past W: never stored)
        const int wc = min(w0 + n, W - 1);
        // (loaded unconditionally, from X when there is no calibration)
        const uintptr_t m = (uintptr_t)0 - (uintptr_t)has_cal;
        const uintptr_t pc = (uintptr_t)(a.nuis + (long long)wc * a.ld_nuis + a.cal_index);
        cv = qfs_load1((const double *)((pc & m) | ((uintptr_t)q.X & ~m)));
    }
    // X by LDS-DMA as well (a compiler-emitted LDS store here would wait for
    // every DMA in flight): waves 0-2 take 128 doubles of the K range each,
    // wave 3 the I panel
    if (wave < 3) {
        if (wave * 128 + 2 * lane < NJ * QF_TILE)
            __builtin_amdgcn_global_load_lds((gbl_void_t *)(q.X + kbase0 + wave * 128 + 2 * lane),
                                             (lds_void_t *)(xs + wave * 128), 16, 0, 0);
    } else if (lane < QF_TILE / 2) {
        __builtin_amdgcn_global_load_lds((gbl_void_t *)(q.X + it.I * QF_TILE + 2 * lane), (lds_void_t *)xI, 16, 0,
                                         0);
    }
    unsigned abase[4];
#pragma unroll
    for (int u = 0; u < 4; u++) abase[u] = lds_addr(smem + li * BK + (((lk * 4 + u) ^ swz(li)) * 2));
    const double *Srow = Sw0 + (size_t)(16 * wave + li) * Np + kbase0 + 8 * lk;
    f64x2 sv[2][4];
    dma_tile(smem, Arow, Np, kbase0, wave, lane);
    qfs_load4(Srow, sv[0]);
    double c2 = 1.0, rc2 = 1.0;
    f64x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; t++) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    auto step = [&](int s, f64x2 (&sv)[4], f64x2 (&sv_next)[4]) {
        // step s's operands, the only loads in flight (the sums pass through the
        // wait, so nothing reads them before it)
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(sv[0]), "+v"(sv[1]), "+v"(sv[2]), "+v"(sv[3]) :: "memory");
        if (s == 0) {
            asm volatile("" : "+v"(cv));
            const double cl = has_cal ? cv : 1.0;
            c2 = cl * cl;
            rc2 = 1.0 / c2;
        }
        // every wave's DMA for step s landed; every wave's reads of step s - 1 done
        // (the asm reads wait for themselves)
        __builtin_amdgcn_s_barrier();
        double2 b[4];
        {
            f64x2 x[4];
            qfs_x_reads(lds_addr(xs + s * BK + 8 * lk), x);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                b[u].x = x[u].x - div_rn(sv[u].x, c2, rc2);
                b[u].y = x[u].y - div_rn(sv[u].y, c2, rc2);
            }
        }
        // the next step's A tile and sums, or at the last step the Delta_I rows
        // into the two buffers the K loop no longer needs
        if (s + 1 < nsteps) {
            dma_next(smem + ((s + 1) % QFS_NBUF) * QFS_BUF_D, true, Arow, kbase0 + (s + 1) * BK, Sw0, 0, 0, Np, wave,
                     lane);
            qfs_load4(Srow + (s + 1) * BK, sv_next);
        } else {
            dma_next(smem + ((s + 1) % QFS_NBUF) * QFS_BUF_D, false, Arow, 0, Sw0, it.I * QF_TILE, 0, Np, wave, lane);
            dma_next(smem + ((s + 2) % QFS_NBUF) * QFS_BUF_D, false, Arow, 0, Sw0, it.I * QF_TILE, 1, Np, wave, lane);
        }
        const unsigned boff = (s % QFS_NBUF) * QFS_BUF_D * 8;
        const unsigned ab[4] = {abase[0] + boff, abase[1] + boff, abase[2] + boff, abase[3] + boff};
#pragma unroll
        for (int u = 0; u < 4; u++) {
            f64x2 af[4];
            switch (u) {   // (the asm operand must be a constant register index)
            case 0: qfs_a_reads<0>(ab, af); break;
            case 1: qfs_a_reads<1>(ab, af); break;
            case 2: qfs_a_reads<2>(ab, af); break;
            default: qfs_a_reads<3>(ab, af); break;
            }
#pragma unroll
            for (int t = 0; t < 4; t++)
                acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[t].x, b[u].x, acc[t], 0, 0, 0);
#pragma unroll
            for (int t = 0; t < 4; t++)
                acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[t].y, b[u].y, acc[t], 0, 0, 0);
        }
    };
#pragma unroll
    for (int s = 0; s < nsteps; s++) {
        step(s, sv[s & 1], sv[(s + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);     // steps not interleaved: the register budget is one step's
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                            // both Delta_I halves landed
    // lane (li, lk)'s walker n takes Delta_I[n][16 t + lk + 4 r] in quadform_body's
    // order; half h of the rows sits in buffer (nsteps + h) % 3
    const double *raw = smem + ((nsteps + (n >> 5)) % QFS_NBUF) * QFS_BUF_D + (n & 31) * QF_TILE;
    const bool live = w0 + n < W;
    double sacc = 0.0;
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int c = 16 * t + lk + 4 * r;
            const double sv = raw[(((c >> 1) ^ (n & 15)) << 1) | (c & 1)];
            const double d = live ? xI[c] - div_rn(sv, c2, rc2) : 0.0;
            sacc += acc[t][r] * d;
        }
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

// The quadratic form's K loop with the compiler's own loads and waits (its
// LDS-DMA wait is vmcnt(0) per step) and the Delta_I rows loaded after it:
// the middle launches, and items wider than two column blocks.
static constexpr int QFSL_TILE_D = QF_TILE * (QF_TILE + 2);
static_assert(QFSL_TILE_D + QF_TILE + QF_MAXKB * QF_TILE + QF_TILE <= QFS_LDS_DOUBLES, "the loop body's LDS");
template <bool SIGNAL>
__device__ __forceinline__ void qfs_body_loop(double *smem, int item_ix, int tile, const QFSArgs &a)
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
    double *c2s = smem + QFSL_TILE_D;            // [64] cal^2 of the tile's walkers
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

// DI_AHEAD: the accept-only launch (qfs_body_nj where the item allows)
template <bool SIGNAL, bool DI_AHEAD>
__device__ __forceinline__ void qfs_body(double *smem, int item_ix, int tile, const QFSArgs &a)
{
    const int nJ = a.src.items[item_ix].nJ;
    if (DI_AHEAD && nJ == 1)
        qfs_body_nj<1, SIGNAL>(smem, item_ix, tile, a);
    else if (DI_AHEAD && nJ == 2)
        qfs_body_nj<2, SIGNAL>(smem, item_ix, tile, a);
    else
        qfs_body_loop<SIGNAL>(smem, item_ix, tile, a);
}

}  // namespace cmamd
