// Native plik_lite likelihood (reference TPlikLiteLikelihood, source/CMB.f90:30-329)
// batched over W walkers on MI355X (gfx950).
//
// Per walker:  cl_b  = sum_{l in bin b} D_l w_l          (CMB.f90:315-325)
//              Delta = X - cl / cal^2                    (CMB.f90:326)
//              -lnL  = Delta^T C^-1 Delta / 2            (CMB.f90:327, Matrix_QuadForm)
//
// Kernels (one launch each, same stream):
//   plik_bin_delta      one workgroup per walker: the walker's D_l rows are
//                       streamed once from HBM (coalesced) into LDS as D_l*w_l
//                       products, then every bin is a contiguous LDS sum.
//                       Writes Delta[w][Np] (Np = nused rounded up to 64).
//   plik_quadform_pairs C^-1 is split into 64x64 blocks; only the upper block
//                       triangle (I <= J) is visited (C^-1 symmetric), one
//                       workgroup per (block pair, 64-walker tile).  T =
//                       C_IJ Delta_J^T on the f64 MFMA (v_mfma_f64_16x16x4f64),
//                       then the column dot with Delta_I and x2 off-diagonal.
//                       Writes partial[pair][w].
//   plik_finalize       -lnL[w] = sum_pair partial[pair][w] / 2, fixed order.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <functional>

#include "common.h"

namespace cmamd {

typedef double f64x4 __attribute__((ext_vector_type(4)));

static constexpr int TILE = 64;          // C^-1 block edge and walker tile

// ------------------------------------------------------------------ kernels

struct BinInfo {
    int field;   // 0 TT, 1 TE, 2 EE  (Theory%Cls (1,1) (2,1) (2,2))
    int lmin;    // absolute l
    int lmax;
    int pad;
};

struct Item {     // one workgroup's share of the symmetric quadratic form
    int I;        // row block (64 rows of C^-1)
    int J0, nJ;   // column blocks J0 .. J0+nJ-1, all >= I
    int pad;
};

struct FieldRanges {   // per used field: l range staged in LDS (even-aligned)
    int lo[3], hi[3], off[3];
};

// Binning + residual.  One workgroup per walker: the walker's TT/TE/EE D_l
// rows are read once (16-byte loads when the layout allows), multiplied by the
// plik weights and kept in LDS; each thread then sums whole bins in l order
// (the reference's dot_product order) and writes Delta = X - cl / cal^2.
// Block 0 also zeroes the split-K arrival counters of the quadratic-form
// kernel that follows on the same stream.
__global__ __launch_bounds__(256) void plik_bin_delta(
    const double *__restrict__ dl, long long ld_field, long long ld_walker,
    const double *__restrict__ nuis, long long ld_nuis,
    const double *__restrict__ wts,          // by absolute l, zero outside the bins
    const BinInfo *__restrict__ bins, const double *__restrict__ X,
    int nused, int Np, FieldRanges fr, int vec_ok,
    double *__restrict__ delta, unsigned int *__restrict__ counters, int n_counters)
{
    extern __shared__ __attribute__((aligned(16))) double prod[];
    const int w = blockIdx.x;
    const int tid = threadIdx.x;
    if (w == 0)
        for (int i = tid; i < n_counters; i += blockDim.x) counters[i] = 0u;
    const double *D = dl + (long long)w * ld_walker;
#pragma unroll
    for (int f = 0; f < 3; f++) {
        const int lo = fr.lo[f], hi = fr.hi[f];
        if (hi < lo) continue;
        const double *Df = D + f * ld_field;
        double *P = prod + fr.off[f] - lo;
        if (vec_ok) {
            // lo is even; pairs (l, l+1), l <= hi (hi odd after alignment)
#pragma unroll 4
            for (int l = lo + 2 * tid; l <= hi; l += 2 * blockDim.x) {
                const double2 d = *reinterpret_cast<const double2 *>(Df + l);
                const double2 q = *reinterpret_cast<const double2 *>(wts + l);
                *reinterpret_cast<double2 *>(P + l) = make_double2(d.x * q.x, d.y * q.y);
            }
        } else {
            const int hs = hi < ld_field ? hi : (int)ld_field - 1;   // never read past the row
#pragma unroll 4
            for (int l = lo + tid; l <= hs; l += blockDim.x) P[l] = Df[l] * wts[l];
        }
    }
    __syncthreads();
    const double cal = nuis[(long long)w * ld_nuis];
    const double c2 = cal * cal;
    double *out = delta + (long long)w * Np;
    for (int i = tid; i < Np; i += blockDim.x) {
        double d = 0.0;
        if (i < nused) {
            const BinInfo b = bins[i];
            const double *p = prod + fr.off[b.field] - fr.lo[b.field];
            double acc = 0.0;
            for (int l = b.lmin; l <= b.lmax; l++) acc += p[l];
            d = X[i] - acc / c2;
        }
        out[i] = d;
    }
}

static constexpr int BK = 32;            // k depth staged per pipeline step (16 chunks of 16 B per row)

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) const void gbl_void_t;

// LDS image of a 64-row x BK-double operand tile: rows of 256 B, unpadded;
// the 16-byte chunk c of row r lives at physical chunk c ^ swz(r).  The
// swizzle makes both the LDS-DMA fill (linear 1 KB pieces) and the MFMA
// fragment reads (ds_read_b128, 8 consecutive k per lane) bank-conflict free.
__device__ __forceinline__ int swz(int r) { return ((r >> 2) & 3) | ((r & 3) << 2); }

// Fill one 64 x BK tile: rows row0..row0+63 of a row-major matrix (stride ld
// doubles), columns k0..k0+BK-1.  4 waves x 4 instructions of 1 KB; lane l
// of instruction j writes LDS bytes [l*16, l*16+16) of piece j = physical
// chunk (l & 15) of row 4j + (l >> 4), so it loads the logical chunk
// (l & 15) ^ swz(row) from global memory.
__device__ __forceinline__ void dma_tile(double *lds_tile, const double *g, size_t ld, int k0, int wave, int lane)
{
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int piece = wave * 4 + q;                 // 0..15, 4 rows each
        const int r = piece * 4 + (lane >> 4);
        const int lc = (lane & 15) ^ swz(r);
        const double *src = g + (size_t)r * ld + k0 + lc * 2;
        __builtin_amdgcn_global_load_lds((gbl_void_t *)src, (lds_void_t *)(lds_tile + piece * 4 * BK), 16, 0, 0);
    }
}

// Quadratic form, symmetric split-K.  With Ct = C^-1 whose diagonal 64x64
// blocks are halved,  Delta^T C^-1 Delta / 2 = sum_I Delta_I^T sum_{J>=I} Ct_IJ Delta_J,
// so -lnL needs only the upper block triangle.  A workgroup owns one
// (row block I, column-block range) item for 64 walkers: a double-buffered
// K loop (LDS-DMA fills one BK step ahead) of f64 MFMA 16x16x4 into four
// 16x16 accumulators per wave, then the dot with Delta_I.  Within a BK step
// lane group g = lane>>4 takes k = 8g .. 8g+7 (any k order is valid as long
// as A and B agree), so each lane reads its fragments as ds_read_b128.
// Partials are handed off in-launch: the last workgroup of each walker tile
// (agent-scope release / ticket / acquire, cdna_hip_programming.md section 5
// split-K recipe) sums them in fixed item order: deterministic results.
__global__ __launch_bounds__(256, 2) void plik_quadform_ksplit(
    const double *__restrict__ Ct, int Np, const double *__restrict__ delta, int W,
    const Item *__restrict__ items, int n_items, int xcd_map,
    double *__restrict__ partial, unsigned int *__restrict__ counters, double *__restrict__ out)
{
    __shared__ __attribute__((aligned(16))) double smem[2 * 2 * TILE * BK];   // [buf][A|B][64][BK], 64 KB
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, lk = lane >> 4;
    // XCD-aware placement: blocks b and b+8 share an XCD; give each XCD whole
    // walker tiles so a tile's Delta stays in one L2 (speed only)
    int item_ix = blockIdx.x, tile = blockIdx.y;
    if (xcd_map) {
        const int b = blockIdx.x + blockIdx.y * gridDim.x;
        const int x = b & 7, j = b >> 3;
        tile = x + 8 * (j / n_items);
        item_ix = j % n_items;
    }
    const Item it = items[item_ix];
    const int w0 = tile * TILE;
    const int nsteps = it.nJ * (TILE / BK);
    const int kbase0 = it.J0 * TILE;
    const double *Arow = Ct + (size_t)(it.I * TILE) * Np;      // rows of the I panel
    const double *Brow = delta + (size_t)w0 * Np;               // walker rows of the tile

    f64x4 acc[4];
#pragma unroll
    for (int t = 0; t < 4; t++) acc[t] = f64x4{0.0, 0.0, 0.0, 0.0};
    dma_tile(smem, Arow, Np, kbase0, wave, lane);
    dma_tile(smem + TILE * BK, Brow, Np, kbase0, wave, lane);
    for (int s = 0; s < nsteps; s++) {
        const int buf = s & 1;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();                              // tile s landed for every wave; buf^1 free
        if (s + 1 < nsteps) {
            double *nb = smem + (buf ^ 1) * 2 * TILE * BK;
            dma_tile(nb, Arow, Np, kbase0 + (s + 1) * BK, wave, lane);
            dma_tile(nb + TILE * BK, Brow, Np, kbase0 + (s + 1) * BK, wave, lane);
        }
        const double *A = smem + buf * 2 * TILE * BK;
        const double *B = A + TILE * BK;
        double2 a[4][4], b[4];
        {
            const int r = 16 * wave + li;
#pragma unroll
            for (int q = 0; q < 4; q++)
                b[q] = *reinterpret_cast<const double2 *>(B + r * BK + (((lk * 4 + q) ^ swz(r)) * 2));
        }
#pragma unroll
        for (int t = 0; t < 4; t++) {
            const int r = 16 * t + li;
#pragma unroll
            for (int q = 0; q < 4; q++)
                a[t][q] = *reinterpret_cast<const double2 *>(A + r * BK + (((lk * 4 + q) ^ swz(r)) * 2));
        }
#pragma unroll
        for (int q = 0; q < 4; q++)
#pragma unroll
            for (int t = 0; t < 4; t++) {
                acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t][q].x, b[q].x, acc[t], 0, 0, 0);
                acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t][q].y, b[q].y, acc[t], 0, 0, 0);
            }
    }
    __syncthreads();                                  // all waves done with the operand buffers
    // Delta_I tile: smem[n][i] (row stride TILE+2)
    for (int e = tid; e < TILE * TILE / 2; e += 256) {
        const int r = e >> 5, c2 = (e & 31) * 2;
        const int w = w0 + r;
        double2 v = *reinterpret_cast<const double2 *>(delta + (size_t)w * Np + it.I * TILE + c2);
        if (w >= W) v = make_double2(0.0, 0.0);
        *reinterpret_cast<double2 *>(smem + r * (TILE + 2) + c2) = v;
    }
    __syncthreads();
    // f64 16x16x4 C/D layout: col = lane&15 (walker n), row = (lane>>4) + 4*r (i)
    const int n = 16 * wave + li;
    double sacc = 0.0;
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int r = 0; r < 4; r++) sacc += acc[t][r] * smem[n * (TILE + 2) + 16 * t + lk + 4 * r];
    sacc += __shfl_xor(sacc, 16);
    sacc += __shfl_xor(sacc, 32);
    double *tile_part = partial + (size_t)tile * n_items * TILE;
    if (lk == 0) tile_part[(size_t)item_ix * TILE + n] = sacc;

    // ---- in-launch hand-off of the tile's partials to its last-arriving workgroup
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned int *flag = reinterpret_cast<unsigned int *>(smem + 64 * (TILE + 2));
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned int t = __hip_atomic_fetch_add(counters + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        flag[0] = (t == (unsigned int)n_items - 1u) ? 1u : 0u;
    }
    __syncthreads();
    if (flag[0] == 0u) return;
    if (tid == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // four item groups per walker, combined in fixed order
    const int g = tid >> 6;
    double part = 0.0;
    for (int k = g; k < n_items; k += 4) part += tile_part[(size_t)k * TILE + lane];
    double *red = smem + 64 * (TILE + 2) + 8;
    red[g * TILE + lane] = part;
    __syncthreads();
    if (tid < TILE) {
        const double v = ((red[lane] + red[TILE + lane]) + red[2 * TILE + lane]) + red[3 * TILE + lane];
        if (w0 + lane < W) out[w0 + lane] = v;
        if (lane == 0) counters[tile] = 0u;
    }
}

// clik packing (cliklike.f90:138-163) -> D_l fields TT, TE, EE for the native kernel
__global__ void clik_to_dl(const double *__restrict__ clp, long long ld, int lmax_tt, int lmax_ee,
                           int lmax_bb, int lmax_te, double *__restrict__ dl, long long ld_field,
                           long long ld_walker, int lmax_out)
{
    const int w = blockIdx.y;
    const double *row = clp + (long long)w * ld;
    const long long o_tt = 0, o_ee = o_tt + lmax_tt + 1, o_bb = o_ee + lmax_ee + 1, o_te = o_bb + lmax_bb + 1;
    for (int l = blockIdx.x * blockDim.x + threadIdx.x; l <= lmax_out; l += gridDim.x * blockDim.x) {
        const double f = l >= 2 ? (double)l * (l + 1) / (2.0 * 3.14159265358979323846264338328) : 0.0;
        double *o = dl + (long long)w * ld_walker;
        o[l] = (l <= lmax_tt) ? row[o_tt + l] * f : 0.0;
        o[ld_field + l] = (l <= lmax_te) ? row[o_te + l] * f : 0.0;
        o[2 * ld_field + l] = (l <= lmax_ee) ? row[o_ee + l] * f : 0.0;
    }
}

// ------------------------------------------------------------------ host side

// Cholesky inverse of an SPD matrix (Matrix_Inverse: dpotrf 'L' + dpotri,
// source/Matrix_utils_new.f90:1478-1569), row-major, in place.
static void spd_inverse(std::vector<double> &A, int n) {
    for (int i = 0; i < n; i++)
        if (std::fabs(A[(size_t)i * n + i]) < 1e-30) fail(CMBL_ERR_NUMERIC, "Matrix_Inverse: very small diagonal");
    for (int j = 0; j < n; j++) {
        double d = A[(size_t)j * n + j];
        for (int k = 0; k < j; k++) d -= A[(size_t)j * n + k] * A[(size_t)j * n + k];
        if (!(d > 0.0)) fail(CMBL_ERR_NUMERIC, "Matrix_Inverse: covariance not positive definite (%d)", j + 1);
        d = std::sqrt(d);
        A[(size_t)j * n + j] = d;
        for (int i = j + 1; i < n; i++) {
            double s = A[(size_t)i * n + j];
            for (int k = 0; k < j; k++) s -= A[(size_t)i * n + k] * A[(size_t)j * n + k];
            A[(size_t)i * n + j] = s / d;
        }
    }
    for (int j = 0; j < n; j++) {           // L^-1, lower
        A[(size_t)j * n + j] = 1.0 / A[(size_t)j * n + j];
        for (int i = j + 1; i < n; i++) {
            double s = 0.0;
            for (int k = j; k < i; k++) s += A[(size_t)i * n + k] * A[(size_t)k * n + j];
            A[(size_t)i * n + j] = -s / A[(size_t)i * n + i];
        }
    }
    std::vector<double> T((size_t)n * n);
    for (int i = 0; i < n; i++)
        for (int j = 0; j <= i; j++) {
            double s = 0.0;
            for (int k = i; k < n; k++) s += A[(size_t)k * n + i] * A[(size_t)k * n + j];
            T[(size_t)i * n + j] = s;
            T[(size_t)j * n + i] = s;
        }
    A.swap(T);
}

static std::vector<double> flat(const std::vector<std::vector<double>> &m) {
    std::vector<double> v;
    for (auto &r : m) v.insert(v.end(), r.begin(), r.end());
    return v;
}

// Fortran unformatted sequential record holding an n x n column-major matrix
// (CMB.f90:236-245: read(lun) cov, then upper -> lower symmetrisation)
static std::vector<double> read_fortran_binary_matrix(const std::string &path, int n) {
    std::ifstream f(path, std::ios::binary);
    if (!f) fail(CMBL_ERR_IO, "cannot read %s", path.c_str());
    int32_t marker = 0;
    f.read(reinterpret_cast<char *>(&marker), 4);
    std::vector<double> colmajor((size_t)n * n);
    if ((size_t)marker != colmajor.size() * 8)
        fail(CMBL_ERR_FORMAT, "%s: record length %d != %d x %d doubles", path.c_str(), marker, n, n);
    f.read(reinterpret_cast<char *>(colmajor.data()), (std::streamsize)(colmajor.size() * 8));
    if (!f) fail(CMBL_ERR_FORMAT, "%s: short record", path.c_str());
    std::vector<double> rm((size_t)n * n);
    for (int i = 0; i < n; i++)            // cov(i,j) = colmajor[j*n+i]; keep upper (i<=j)
        for (int j = i; j < n; j++) {
            double v = colmajor[(size_t)j * n + i];
            rm[(size_t)i * n + j] = v;
            rm[(size_t)j * n + i] = v;
        }
    return rm;
}

std::string load_paramnames(const std::string &path, int *count) {
    std::ifstream f(path);
    if (!f) fail(CMBL_ERR_IO, "cannot read paramnames %s", path.c_str());
    std::string line, names;
    int n = 0;
    while (std::getline(f, line)) {
        auto t = split_ws(line);
        if (t.empty() || t[0][0] == '#') continue;
        std::string nm = t[0];
        if (!nm.empty() && nm.back() == '*') nm.pop_back();   // derived marker
        names += (n ? " " : "") + nm;
        n++;
    }
    *count = n;
    return names;
}

struct PlikLite final : Like {
    static constexpr int plmin = 30;     // CMB.f90:33
    static constexpr int nbins_total = 613;
    const int nbincl[3] = {215, 199, 199};
    int nused = 0, Np = 0, nblk = 0, lmax_needed = 0;
    FieldRanges fr{};
    int lds_doubles = 0;
    DevBuf d_wts, d_bins, d_X, d_invcov;
    // work-item lists for column-block chunk sizes KB = 1..MAXKB
    static constexpr int MAXKB = 5;
    DevBuf d_items[MAXKB + 1];
    std::vector<Item> items[MAXKB + 1];
    std::map<int, int> kb_for_tiles;
    DevBuf conv;   // clik -> D_l staging

    explicit PlikLite(const Ini &ini) {
        tag = "PLIK_LITE";
        name = ini.str("name");
        if (name.empty()) {
            std::string fn = ini.filename();
            size_t s = fn.find_last_of('/');
            fn = fn.substr(s == std::string::npos ? 0 : s + 1);
            size_t d = fn.find_last_of('.');
            name = d == std::string::npos ? fn : fn.substr(0, d);
        }
        nuisance_names = load_paramnames(ini.relative_filename("calibration_param", true), &n_nuis);
        std::string use_cl = ini.str("use_cl");
        auto dat = load_txt(ini.relative_filename("data", true));
        auto blmin = flat(load_txt(ini.relative_filename("blmin", true)));
        auto blmax = flat(load_txt(ini.relative_filename("blmax", true)));
        auto wfile = flat(load_txt(ini.relative_filename("weights", true)));
        if ((int)dat.size() < nbins_total || dat[0].size() < 2)
            fail(CMBL_ERR_FORMAT, "plik_lite data file must have >= %d rows of >= 2 columns", nbins_total);
        int maxbin = nbincl[0];
        if ((int)blmin.size() < maxbin || (int)blmax.size() < maxbin)
            fail(CMBL_ERR_FORMAT, "plik_lite blmin/blmax need %d entries", maxbin);
        std::vector<int> bmin(maxbin), bmax(maxbin);
        for (int i = 0; i < maxbin; i++) {
            bmin[i] = (int)blmin[i] + plmin;   // CMB.f90:225-227
            bmax[i] = (int)blmax[i] + plmin;
        }
        const int nw = (int)wfile.size();
        lmax_needed = plmin + nw - 1;
        std::vector<double> wts(lmax_needed + 1, 0.0);
        for (int i = 0; i < nw; i++) {          // CMB.f90:230-233
            double ls = (double)(plmin + i);
            wts[plmin + i] = wfile[i] * (2.0 * 3.14159265358979323846264338328) / ls / (ls + 1.0);
        }
        std::vector<double> cov;
        std::string covb = ini.str("cov_file_binary");
        if (!covb.empty()) {
            cov = read_fortran_binary_matrix(ini.relative_filename("cov_file_binary", true), nbins_total);
        } else {
            cov = flat(load_txt(ini.relative_filename("cov_file", true)));
            if (cov.size() != (size_t)nbins_total * nbins_total)
                fail(CMBL_ERR_FORMAT, "plik_lite cov_file must be %d x %d", nbins_total, nbins_total);
        }
        // bins_for_L_range (CMB.f90:250-263)
        std::vector<int> usebins;
        bool ranged = false;
        std::string rng = ini.str("bins_for_L_range");
        if (!rng.empty()) {
            auto t = split_ws(rng);
            if (t.size() < 2) fail(CMBL_ERR_FORMAT, "bins_for_L_range needs two integers");
            int rmin = std::stoi(t[0]), rmax = std::stoi(t[1]);
            int mb = std::max(nbincl[0], std::max(nbincl[1], nbincl[2]));
            for (int i = 1; i <= mb; i++) {
                double c = (bmin[i - 1] + bmax[i - 1]) / 2.0;
                if (rmin <= c && c <= rmax) usebins.push_back(i);
            }
            ranged = true;
        }
        const char *names[3] = {"TT", "TE", "EE"};
        auto toks = split_ws(use_cl);
        std::vector<int> used_idx;
        std::vector<BinInfo> binfo;
        int offset = 0;
        for (int s = 0; s < 3; s++) {          // CMB.f90:265-297
            bool used = false;
            for (auto &t : toks) used |= (t == names[s]);
            if (used) {
                std::vector<int> bl;
                if (ranged) {
                    for (int b : usebins) if (b <= nbincl[s]) bl.push_back(b);
                } else {
                    for (int b = 1; b <= nbincl[s]; b++) bl.push_back(b);
                }
                int mx = 0;
                for (int b : bl) {
                    used_idx.push_back(b + offset - 1);
                    binfo.push_back({s, bmin[b - 1], bmax[b - 1], 0});
                    mx = std::max(mx, bmax[b - 1]);
                }
                const int ij[3][2] = {{1, 1}, {2, 1}, {2, 2}};
                cl_lmax[(ij[s][0] - 1) * 4 + (ij[s][1] - 1)] = mx;
            }
            offset += nbincl[s];
        }
        nused = (int)used_idx.size();
        if (nused == 0) fail(CMBL_ERR_FORMAT, "plik_lite: use_cl selects no bins");
        for (auto &b : binfo)
            if (b.lmin < plmin || b.lmax > lmax_needed) fail(CMBL_ERR_FORMAT, "plik_lite: bin outside weights range");
        std::vector<double> X(nused), ic((size_t)nused * nused);
        for (int i = 0; i < nused; i++) {       // CMB.f90:298-299
            X[i] = dat[used_idx[i]][1];
            for (int j = 0; j < nused; j++) ic[(size_t)i * nused + j] = cov[(size_t)used_idx[i] * nbins_total + used_idx[j]];
        }
        spd_inverse(ic, nused);                 // CMB.f90:300

        // device layout
        Np = (nused + TILE - 1) / TILE * TILE;
        nblk = Np / TILE;
        // Ct: C^-1 padded to Np with the diagonal 64x64 blocks halved (exact: x0.5)
        std::vector<double> icp((size_t)Np * Np, 0.0), Xp(Np, 0.0);
        for (int i = 0; i < nused; i++) {
            Xp[i] = X[i];
            for (int j = 0; j < nused; j++) {
                const double v = ic[(size_t)i * nused + j];
                icp[(size_t)i * Np + j] = (i / TILE == j / TILE) ? 0.5 * v : v;
            }
        }
        for (int kb = 1; kb <= MAXKB; kb++)
            for (int I = 0; I < nblk; I++)
                for (int J0 = I; J0 < nblk; J0 += kb) items[kb].push_back(Item{I, J0, std::min(kb, nblk - J0), 0});
        // LDS ranges per field, widened to even start / odd end for 16-byte access
        lds_doubles = 0;
        for (int f = 0; f < 3; f++) {
            fr.lo[f] = 1 << 30;
            fr.hi[f] = -1;
        }
        for (auto &b : binfo) {
            fr.lo[b.field] = std::min(fr.lo[b.field], b.lmin);
            fr.hi[b.field] = std::max(fr.hi[b.field], b.lmax);
        }
        for (int f = 0; f < 3; f++) {
            fr.off[f] = lds_doubles;
            if (fr.hi[f] >= fr.lo[f]) {
                fr.lo[f] &= ~1;
                fr.hi[f] |= 1;
                lds_doubles += fr.hi[f] - fr.lo[f] + 1;
            } else {
                fr.lo[f] = 0;
                fr.hi[f] = -1;
            }
        }

        binfo.resize(Np, BinInfo{0, 1, 0, 0});
        int wmax = lmax_needed;
        for (int f = 0; f < 3; f++) wmax = std::max(wmax, fr.hi[f]);
        wts.resize((size_t)wmax + 2, 0.0);
        d_wts.alloc(wts.size() * 8);
        d_wts.upload(wts.data(), wts.size() * 8);
        d_bins.alloc(binfo.size() * sizeof(BinInfo));
        d_bins.upload(binfo.data(), binfo.size() * sizeof(BinInfo));
        d_X.alloc(Xp.size() * 8);
        d_X.upload(Xp.data(), Xp.size() * 8);
        d_invcov.alloc(icp.size() * 8);
        d_invcov.upload(icp.data(), icp.size() * 8);
        for (int kb = 1; kb <= MAXKB; kb++) {
            d_items[kb].alloc(items[kb].size() * sizeof(Item));
            d_items[kb].upload(items[kb].data(), items[kb].size() * sizeof(Item));
        }
        const size_t lds = (size_t)lds_doubles * 8;
        if (lds > 64 * 1024)
            HIP_CHECK(hipFuncSetAttribute((const void *)plik_bin_delta,
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    }

    static int wpad(int W) { return (W + TILE - 1) / TILE * TILE; }

    // Column-block chunk per work item: the largest chunk whose longest-first
    // greedy schedule over 2 workgroups/CU x 256 CUs is (near) the fastest,
    // counting a fixed per-workgroup overhead of half a block.
    int choose_kb(int tiles) {
        auto itk = kb_for_tiles.find(tiles);
        if (itk != kb_for_tiles.end()) return itk->second;
        const int slots = 512;
        int best_kb = 1;
        double best = 1e300;
        for (int kb = 1; kb <= MAXKB; kb++) {
            std::vector<double> load(slots, 0.0);
            std::vector<double> jobs;
            for (auto &x : items[kb])
                for (int t = 0; t < tiles; t++) jobs.push_back(x.nJ + 0.5);
            std::sort(jobs.begin(), jobs.end(), std::greater<double>());
            for (double j : jobs) *std::min_element(load.begin(), load.end()) += j;
            const double makespan = *std::max_element(load.begin(), load.end()) + 0.02 * items[kb].size();
            if (makespan < best * 0.98) {
                best = makespan;
                best_kb = kb;
            }
        }
        kb_for_tiles[tiles] = best_kb;
        return best_kb;
    }

    size_t workspace_size(int W) const override {
        const size_t Wp = (size_t)wpad(W), tiles = Wp / TILE;
        size_t nmax = 0;
        for (int kb = 1; kb <= MAXKB; kb++) nmax = std::max(nmax, items[kb].size());
        return (Wp * Np + tiles * nmax * TILE) * sizeof(double) + ((tiles * 4 + 255) & ~size_t(255));
    }

    void loglike_batch(int W, const double *dl, long long ld_field, long long ld_walker,
                       const double *nuis, long long ld_nuis, double *out, void *ws,
                       hipStream_t stream) override {
        if (W <= 0) return;
        if (n_nuis < 1 || !nuis) fail(CMBL_ERR_ARG, "plik_lite needs the calibration nuisance parameter");
        if (ld_field < lmax_needed + 1) fail(CMBL_ERR_ARG, "ld_field %lld < lmax+1 = %d", ld_field, lmax_needed + 1);
        if (ld_walker < 3 * ld_field) fail(CMBL_ERR_ARG, "ld_walker must cover the TT, TE, EE fields");
        const int Wp = wpad(W), tiles = Wp / TILE;
        if (!ws) {
            own_ws.grow(workspace_size(W));
            ws = own_ws.p;
        }
        const int kb = choose_kb(tiles);
        const int n_items = (int)items[kb].size();
        size_t nmax = 0;
        for (int k = 1; k <= MAXKB; k++) nmax = std::max(nmax, items[k].size());
        double *delta = static_cast<double *>(ws);
        double *partial = delta + (size_t)Wp * Np;
        unsigned int *counters = reinterpret_cast<unsigned int *>(partial + (size_t)tiles * nmax * TILE);
        // 16-byte D_l loads need 16-byte aligned rows and the widened ranges inside each row
        int vec_ok = ((reinterpret_cast<uintptr_t>(dl) & 15) == 0) && (ld_field % 2 == 0) && (ld_walker % 2 == 0);
        for (int f = 0; f < 3; f++)
            if (fr.hi[f] >= fr.lo[f] && fr.hi[f] >= ld_field) vec_ok = 0;
        timed_launch("plik_bin_delta", stream, [&](hipEvent_t e0, hipEvent_t e1) {
            hipExtLaunchKernelGGL(plik_bin_delta, dim3(W), dim3(256), (size_t)lds_doubles * 8, stream, e0, e1, 0, dl, ld_field,
                               ld_walker, nuis, ld_nuis, d_wts.as<double>(), d_bins.as<BinInfo>(), d_X.as<double>(),
                               nused, Np, fr, vec_ok, delta, counters, tiles);
        });
        HIP_CHECK(hipGetLastError());
        timed_launch("plik_quadform_ksplit", stream, [&](hipEvent_t e0, hipEvent_t e1) {
            hipExtLaunchKernelGGL(plik_quadform_ksplit, dim3(n_items, tiles), dim3(256), 0, stream, e0, e1, 0,
                               d_invcov.as<double>(), Np, delta, W, d_items[kb].as<Item>(), n_items,
                               (int)(tiles % 8 == 0), partial, counters, out);
        });
        HIP_CHECK(hipGetLastError());
    }
};

std::unique_ptr<Like> make_plik_lite(const Ini &ini) { return std::unique_ptr<Like>(new PlikLite(ini)); }

// exported for the clik entry point (api.cpp)
void launch_clik_to_dl(const double *clp, long long ld, const int *lm, double *dl, long long ld_field,
                       long long ld_walker, int lmax_out, int W, hipStream_t stream) {
    hipLaunchKernelGGL(clik_to_dl, dim3((lmax_out + 256) / 256, W), dim3(256), 0, stream, clp, ld, lm[0], lm[1],
                       lm[2], lm[3], dl, ld_field, ld_walker, lmax_out);
    HIP_CHECK(hipGetLastError());
}

}  // namespace cmamd
