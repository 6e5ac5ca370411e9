// plik_lite's binning as a device body: plik.hip's plik_bin_delta (Delta =
// X - bin / cal^2 into the quadratic form's rows) and the sampler's bin
// co-run (raw bin sums, no calibration, in the launch that proposes the
// calibrations; sampler.hip mh_bin_kernel).  Reference: TPlikLiteLikelihood
// LogLike, source/CMB.f90:315-326.
#pragma once

#include "common.h"

namespace cmamd {

struct BinInfo {
    int field;   // 0 TT, 1 TE, 2 EE  (Theory%Cls (1,1) (2,1) (2,2))
    int lmin;    // absolute l
    int lmax;
    int pad;
};

struct FieldRanges {   // per used field: l range staged in LDS (even-aligned), its bins [b0, b1)
    int lo[3], hi[3], b0[3], b1[3];
};

struct PlikBinArgs {
    const double *dl;              // theory D_l: field f of walker w at dl + w ld_walker + f ld_field
    long long ld_field, ld_walker;
    const double *wts;             // by absolute l, zero outside the bins
    const BinInfo *bins;
    const double *X;               // [Np] data vector, zero padded
    int nused, Np;
    FieldRanges fr;
    int vec_ok;                    // 16-byte D_l loads
    int lds_doubles;               // the body's LDS (doubles)
};

// One workgroup per (walker w, field f): the field's D_l row is read once
// (16-byte loads when the layout allows), multiplied by the plik weights and
// kept in LDS (plik_bin_products, which ends in a barrier); each thread then
// sums whole bins in l order (the reference's dot_product order) and writes,
// for the field's bins, the raw sum (RAW) or Delta = X - sum / c2 with c2 =
// cal^2 (plik_bin_emit).  rows: [W][Np]; the padding columns are not touched.
// Returns false (nothing staged) when field f is not used.
__device__ __forceinline__ bool plik_bin_products(const PlikBinArgs &a, double *prod, int w, int f)
{
    const int tid = threadIdx.x;
    const int lo = a.fr.lo[f], hi = a.fr.hi[f];
    if (hi < lo) return false;
    const double *Df = a.dl + (long long)w * a.ld_walker + f * a.ld_field;
    double *P = prod - lo;
    if (a.vec_ok) {
        // lo is even, hi odd: pairs (l, l+1)
#pragma unroll 4
        for (int l = lo + 2 * tid; l <= hi; l += 2 * blockDim.x) {
            const double2 d = *reinterpret_cast<const double2 *>(Df + l);
            const double2 q = *reinterpret_cast<const double2 *>(a.wts + l);
            *reinterpret_cast<double2 *>(P + l) = make_double2(d.x * q.x, d.y * q.y);
        }
    } else {
        const int hs = hi < a.ld_field ? hi : (int)a.ld_field - 1;   // never read past the row
#pragma unroll 4
        for (int l = lo + tid; l <= hs; l += blockDim.x) P[l] = Df[l] * a.wts[l];
    }
    __syncthreads();
    return true;
}

template <bool RAW>
__device__ __forceinline__ void plik_bin_emit(const PlikBinArgs &a, const double *prod, int w, int f, double c2,
                                              double *rows)
{
    const double *P = prod - a.fr.lo[f];
    double *out = rows + (long long)w * a.Np;
    for (int i = a.fr.b0[f] + threadIdx.x; i < a.fr.b1[f]; i += blockDim.x) {
        const BinInfo b = a.bins[i];
        double acc = 0.0;
        for (int l = b.lmin; l <= b.lmax; l++) acc += P[l];
        out[i] = RAW ? acc : a.X[i] - acc / c2;
    }
}

template <bool RAW>
__device__ __forceinline__ void plik_bin_body(const PlikBinArgs &a, double *prod, int w, int f, const double *nuis,
                                              long long ld_nuis, double *rows)
{
    if (!plik_bin_products(a, prod, w, f)) return;
    double c2 = 1.0;
    if (!RAW) {
        const double cal = nuis[(long long)w * ld_nuis];
        c2 = cal * cal;
    }
    plik_bin_emit<RAW>(a, prod, w, f, c2, rows);
}

}  // namespace cmamd
