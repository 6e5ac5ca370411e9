// Device body of the fused window pass's vectorised kernel (theorypass.hip),
// shared by theory_window_vec and by the sampler's unified step launch, whose
// workgroups run it beside the quadratic form's and mh_kernel's (sampler.hip,
// mh_step_kernel).  The LDS comes from the caller (tp_vec_lds_bytes).
#pragma once

#include "divrn.h"
#include "theorypass.h"

namespace cmamd {

typedef double f64x4 __attribute__((ext_vector_type(4)));

#ifndef TP_STAMP
#define TP_STAMP(i) ((void)0)
#endif

template <int NB> constexpr int tp_vec_lds_bytes() {
    return 2 * NB * 16 * (32 + 2) * 8 + TP_MAXCOL * (int)sizeof(TPCol) + TP_MAXCOL * 8 + TP_MAXSTEP * 8 +
           TP_MAXSTEP * TP_MAXCOL;
}

// The same pass when every theory row is 16-byte aligned (the sampler's
// case), written so that each step's loads are unconditional straight-line
// code: the theory rows two steps ahead (addresses clamped into the row, l
// past the item read as 0), the weight tiles of every block two steps ahead
// in registers (blocks past the item's own read its neighbour's weights or
// the padding: stored, never used), and the last two steps peeled off.  The
// compiler then counts the loads in flight exactly, and a step waits only for
// its own data instead of draining the prefetch (vmcnt(0)) at the weight
// store, which held every step to a full memory latency.
//
// RAW (the sampler's unified step launch, mh_step_kernel): no calibration at
// all -- every column's sum v is stored as it comes out of the MFMAs, at the
// index its stage's output would take (out is then the stage's raw-sum buffer);
// the consumers apply the calibrations of the step that reads them with the
// emit's own operations (X - v / cal^2 in the quadratic form's operand, v /
// cal^2 in the small chi^2's partial rows), so the results are the same bits.
//
// W2: the weight tiles two steps ahead in two register sets (the standalone
// kernels: theory_window_pair 41.1 -> 40.0 us a launch, the drag step 416.5-417.5
// -> 412.4-415.6 us; in the unified launch, whose registers the other roles
// share, it measured 0.3 us slower: there the one-step form runs)
template <int NB, bool RAW = false, bool W2 = false>
__device__ __forceinline__ void tp_vec_body(const TPDev &c, const double *__restrict__ dl, long long ld_field,
                                            long long ld_walker, int W, char *lds, int b)
{
    constexpr int LPL = 8, STEP = 4 * LPL, NSUB = TP_CHUNK / STEP, WROW = STEP + 2;
    double *wsh = reinterpret_cast<double *>(lds);                                   // [buf][col block][col][l]
    TPCol *csh = reinterpret_cast<TPCol *>(wsh + 2 * NB * 16 * WROW);               // [TP_MAXCOL]
    double *xsh = reinterpret_cast<double *>(csh + TP_MAXCOL);                       // [TP_MAXCOL]
    unsigned long long *esh = reinterpret_cast<unsigned long long *>(xsh + TP_MAXCOL);   // [TP_MAXSTEP]
    unsigned char *msh = reinterpret_cast<unsigned char *>(esh + TP_MAXSTEP);        // [TP_MAXSTEP][TP_MAXCOL]
    const int2 unit = c.units[b];
    const int item = unit.x, tile = unit.y;
    if (item < 0) return;
    TP_STAMP(0);
#ifdef CMAMD_TP_STAMPS
    const unsigned long long rt0_ = __builtin_amdgcn_s_memrealtime();
#endif
    const TPItem it = c.items[item];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, kq = lane >> 4;
    const int w = (c.tile_off + tile) * 64 + wave * 16 + li;
    const int wl = min(w, W - 1);
    const double *Df = dl + (long long)wl * ld_walker + (long long)it.field * ld_field;
    const int lcap = ((int)ld_field - 2) & ~1;
    const int ncb = it.nsb;
    const int nstep = it.nst;
    double tA[LPL], tB[LPL], tC[LPL], a[LPL];
    auto load_t = [&](int st, double *dst) {  // raw rows, addresses clamped into the row
        const int lb = it.l0 + st * STEP + 2 * kq;
#pragma unroll
        for (int q = 0; q < LPL / 2; q++) {
            const double2 v = *reinterpret_cast<const double2 *>(Df + min(lb + 8 * q, lcap));
            dst[2 * q] = v.x;
            dst[2 * q + 1] = v.y;
        }
    };
    const int wc = tid >> 4, wp = 2 * (tid & 15);
    double2 wr0{}, wr1{}, wr2{}, wr3{};      // named registers: an array here lands in scratch
#define TP_WR wr0, wr1, wr2, wr3
    // W2: two named register sets: step st fetches the weights of st + 2 into
    // one while the other holds those of st + 1 (fetched a whole step earlier)
    // for the LDS store at the step's end
    double2 wa0{}, wa1{}, wa2{}, wa3{}, wb0{}, wb1{}, wb2{}, wb3{};
#define TP_WA wa0, wa1, wa2, wa3
#define TP_WB wb0, wb1, wb2, wb3
    auto fetch_w = [&](int st, double2 &r0, double2 &r1, double2 &r2, double2 &r3) {
        const int ch = st / NSUB, sub = st % NSUB;
        const double *base = c.w + it.woff + (long long)ch * ncb * 16 * TP_CHUNK + sub * STEP + wc * TP_CHUNK + wp;
        r0 = *reinterpret_cast<const double2 *>(base);
        r1 = *reinterpret_cast<const double2 *>(base + 16 * TP_CHUNK);
        if constexpr (NB > 2) {
            r2 = *reinterpret_cast<const double2 *>(base + 2 * 16 * TP_CHUNK);
            r3 = *reinterpret_cast<const double2 *>(base + 3 * 16 * TP_CHUNK);
        }
    };
    auto store_w = [&](int buf, const double2 &r0, const double2 &r1, const double2 &r2, const double2 &r3) {
        double *d = wsh + (buf * NB * 16 + wc) * WROW + wp;
        *reinterpret_cast<double2 *>(d) = r0;
        *reinterpret_cast<double2 *>(d + 16 * WROW) = r1;
        if constexpr (NB > 2) {
            *reinterpret_cast<double2 *>(d + 2 * 16 * WROW) = r2;
            *reinterpret_cast<double2 *>(d + 3 * 16 * WROW) = r3;
        }
    };
    auto read_w = [&](int buf, int cb) {
        const double *src = wsh + ((buf * NB + cb) * 16 + li) * WROW + 2 * kq;
#pragma unroll
        for (int q = 0; q < LPL / 2; q++) {
            const double2 v = *reinterpret_cast<const double2 *>(src + 8 * q);
            a[2 * q] = v.x;
            a[2 * q + 1] = v.y;
        }
    };
    f64x4 acc[NB], bcc[NB];
#pragma unroll
    for (int cb = 0; cb < NB; cb++) acc[cb] = bcc[cb] = f64x4{0.0, 0.0, 0.0, 0.0};
    // prologue: theory steps 0, 1; weights of step 0 into LDS, of step 1 in registers
    load_t(0, tA);
    load_t(1, tB);                       // nstep >= 2: an item is whole 64-l chunks
    if constexpr (W2) {
        fetch_w(0, TP_WA);
        fetch_w(1, TP_WB);
    } else {
        fetch_w(0, TP_WR);
    }
    if (tid < it.ncol) {
        const TPCol d = c.cols[it.cdesc + tid];
        csh[tid] = d;
        const int kind = d.out ? c.out[1].kind : c.out[0].kind;
        const double *X = d.out ? c.out[1].X : c.out[0].X;
        xsh[tid] = (kind == 1 && !RAW) ? X[d.row] : 0.0;
    }
    if (tid < nstep) esh[tid] = c.emit[it.soff + tid];
    for (int q = tid; q < nstep * (TP_MAXCOL / 4); q += 256)
        reinterpret_cast<unsigned int *>(msh)[q] =
            reinterpret_cast<const unsigned int *>(c.cmap + (long long)it.soff * TP_MAXCOL)[q];
    double c2[TP_MAXOUT] = {1.0, 1.0}, rc2[TP_MAXOUT] = {1.0, 1.0};   // cal^2 and its reciprocal (div_rn)
    if (!RAW) {
#pragma unroll
        for (int o = 0; o < TP_MAXOUT; o++) {
            const int ci = o ? c.out[1].cal_index : c.out[0].cal_index;
            const double *nu = o ? c.out[1].nuis : c.out[0].nuis;
            const long long ldn = o ? c.out[1].ld_nuis : c.out[0].ld_nuis;
            double cl = 1.0;
            if (ci >= 0 && nu) cl = nu[(long long)wl * ldn + ci];
            c2[o] = cl * cl;
            rc2[o] = 1.0 / c2[o];
        }
    }
    if constexpr (W2)
        store_w(0, TP_WA);
    else
        store_w(0, TP_WR);
    __syncthreads();
    TP_STAMP(1);
    auto emit = [&](int st, unsigned long long e, int cb, f64x4 &a0, f64x4 &b0) {
        int col[4];
        bool on[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int slot = 16 * cb + kq + 4 * r;
            on[r] = (e >> slot) & 1ull;
            col[r] = msh[st * TP_MAXCOL + slot] & (TP_MAXCOL - 1);   // 255 (no column) -> any: not stored
        }
        TPCol d[4];
        double x[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            d[r] = csh[col[r]];
            x[r] = xsh[col[r]];
        }
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const double v = a0[r] + b0[r];
            a0[r] = on[r] ? 0.0 : a0[r];
            b0[r] = on[r] ? 0.0 : b0[r];
            const bool o1 = d[r].out != 0;
            const double q = (!RAW && d[r].cal) ? div_rn(v, o1 ? c2[1] : c2[0], o1 ? rc2[1] : rc2[0]) : v;   // v / cal^2
            if (on[r] && w < W) {
                double *out = o1 ? c.out[1].out : c.out[0].out;
                if ((o1 ? c.out[1].kind : c.out[0].kind) == 0)
                    out[(long long)d[r].row * W + w] = q;
                else
                    out[(long long)w * (o1 ? c.out[1].ld : c.out[0].ld) + d[r].row] = RAW ? v : x[r] - q;
            }
        }
    };
    auto closes = [&](int st) {   // the columns that end at step st
        const unsigned long long e = esh[st];
#pragma unroll
        for (int cb = 0; cb < NB; cb++)
            if ((e >> (16 * cb)) & 0xffffull) emit(st, e, cb, acc[cb], bcc[cb]);
    };
    auto compute = [&](int st, const double *tc, bool tail) {
        double tb[LPL];
        const int lb = it.l0 + st * STEP + 2 * kq;
#pragma unroll
        for (int q = 0; q < LPL / 2; q++)
#pragma unroll
            for (int h = 0; h < 2; h++) tb[2 * q + h] = (!tail || lb + 8 * q + h <= it.l1) ? tc[2 * q + h] : 0.0;
        const int cur = st & 1;
        const unsigned m = (unsigned)(it.act >> (4 * st)) & 15u;
#pragma unroll
        for (int cb = 0; cb < NB; cb++)
            if (m & (1u << cb)) {
                read_w(cur, cb);
#pragma unroll
                for (int s2 = 0; s2 < LPL; s2 += 2) {
                    acc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s2], tb[s2], acc[cb], 0, 0, 0);
                    bcc[cb] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s2 + 1], tb[s2 + 1], bcc[cb], 0, 0, 0);
                }
            }
    };
    int st = 0;
    if constexpr (W2) {
        // main steps: weights of st + 2 and theory of st + 2 in flight; step s's
        // theory lives in buffer s mod 3 (A, B, C), its weights' registers in set
        // s mod 2 (A, B) until stored at step s - 1
        auto step = [&](int st, const double *tc, double *tl, double2 &f0, double2 &f1, double2 &f2, double2 &f3,
                        const double2 &s0, const double2 &s1, const double2 &s2, const double2 &s3) {
            fetch_w(st + 2, f0, f1, f2, f3);
            load_t(st + 2, tl);
            compute(st, tc, false);
            closes(st);
            store_w((st & 1) ^ 1, s0, s1, s2, s3);
            __syncthreads();
        };
        while (st + 2 < nstep) {
            step(st, tA, tC, TP_WA, TP_WB);
            if (++st + 2 >= nstep) break;
            step(st, tB, tA, TP_WB, TP_WA);
            if (++st + 2 >= nstep) break;
            step(st, tC, tB, TP_WA, TP_WB);
            if (++st + 2 >= nstep) break;
            step(st, tA, tC, TP_WB, TP_WA);
            if (++st + 2 >= nstep) break;
            step(st, tB, tA, TP_WA, TP_WB);
            if (++st + 2 >= nstep) break;
            step(st, tC, tB, TP_WB, TP_WA);
            ++st;
        }
        // the last two steps: nothing more to load; step st + 1's weights (set
        // (st + 1) mod 2) go to the buffer step st - 1 read, behind its barrier
        if (st & 1)
            store_w((st & 1) ^ 1, TP_WA);
        else
            store_w((st & 1) ^ 1, TP_WB);
        auto tail = [&](const double *t0, const double *t1) {
            compute(st, t0, true);
            __syncthreads();
            closes(st);
            compute(st + 1, t1, true);
            closes(st + 1);
        };
        switch (st % 3) {
            case 0: tail(tA, tB); break;
            case 1: tail(tB, tC); break;
            default: tail(tC, tA); break;
        }
    } else {
        // main steps: weights of st + 1 and theory of st + 2 in flight; step s
        // lives in buffer s mod 3 (A, B, C)
        auto step = [&](int st, const double *tc, double *tl) {
            fetch_w(st + 1, TP_WR);
            load_t(st + 2, tl);
            compute(st, tc, false);
            closes(st);
            store_w((st & 1) ^ 1, TP_WR);
            __syncthreads();
        };
        while (st + 2 < nstep) {
            step(st, tA, tC);
            if (++st + 2 >= nstep) break;
            step(st, tB, tA);
            if (++st + 2 >= nstep) break;
            step(st, tC, tB);
            ++st;
        }
        // the last two steps: nothing more to load
        auto tail = [&](const double *t0, const double *t1) {
            fetch_w(st + 1, TP_WR);
            compute(st, t0, true);
            store_w((st & 1) ^ 1, TP_WR);
            __syncthreads();
            closes(st);
            compute(st + 1, t1, true);
            closes(st + 1);
        };
        switch (st % 3) {
            case 0: tail(tA, tB); break;
            case 1: tail(tB, tC); break;
            default: tail(tC, tA); break;
        }
    }
#undef TP_WR
#undef TP_WA
#undef TP_WB
    TP_STAMP(2);
#ifdef CMAMD_TP_STAMPS
    if (threadIdx.x == 0 && b < 4096) {
        g_tp_stamps[b][4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        g_tp_stamps[b][5] = __builtin_amdgcn_s_getreg((3 << 11) | 20);
        g_tp_stamps[b][6] = item;
        g_tp_stamps[b][7] = (unsigned long long)nstep * 1000 + __builtin_popcountll(it.act);
    }
#endif
    TP_STAMP(3);
#ifdef CMAMD_TP_STAMPS
    const unsigned long long rt1_ = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && b < 4096) {
        g_tp_stamps[b][8] = rt0_;
        g_tp_stamps[b][9] = rt1_;
    }
#endif
}

}  // namespace cmamd
