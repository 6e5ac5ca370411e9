// Fused window pass (see theorypass.h).
//
// A work item is an l range of one theory field with up to 64 columns from
// any of the stages (four 16-column MFMA blocks); a workgroup takes one item
// for 64 walkers and walks the range in 32-l steps.  The contraction is
// cmbl_window_direct's (cmblikes.hip): lane (walker li, quarter kq) holds the 8
// l {l0 + 32 st + 8 j + 2 kq + h : j < 4, h < 2} of its walker's row in slot
// 2 j + h (16-byte loads, two steps ahead of the MFMAs), and MFMA step
// s = 2 j + h contracts the four l {8 j + 2 kq + h} against the weights, which
// the block's four waves share through a double-buffered LDS tile.  Columns
// are ordered wide first (CMBlikes windows), then plik bins by l, and a block
// runs only in the steps where it has weight.
// Each column's sum goes to its stage: a CMBlikes partial row (/ cal^2 for
// calibrated map pairs, AdaptTheoryForMaps CMBlikes.f90:1113-1124), or plik's
// Delta = X - sum / cal^2 (CMB.f90:315-326; the bin sum in MFMA order, not the
// reference's l order: rtol 1e-12 against plik_bin_delta).  No column
// straddles two items, so every output is one workgroup's store.
//
// Slots: the columns of an item are dealt to the 16-column MFMA blocks' slots
// by their step ranges (interval colouring), so a plik bin takes a slot only
// for the steps it covers, and its sum is written (and the slot zeroed) right
// after the MFMAs of its last step.  The lensing windows (9 slots, every step)
// and the few plik bins open in one 32-l step then share one block: one
// active block per step instead of two (act 16 -> 8 on the long TT/TE/EE
// items), 26.2 -> 24.2 us.
//
// Measured (MI355X, W = 1024, plik_lite + lensing): 24.2 us against 30 us for
// plik_bin_delta + cmbl_window_direct.  Summing the bins on the VALU from an
// LDS copy of the tile instead (the reference's order) took 39-42 us.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>

#include "divrn.h"
#include "theorypass.h"

namespace cmamd {

typedef double f64x4 __attribute__((ext_vector_type(4)));

#ifdef CMAMD_STAMPS
#define CMAMD_TP_STAMPS
// per block of the last launch: s_memtime at start, after the prologue, after
// the step loop, at the end; HW_ID, XCC_ID and the item (tools/tp_stamps.py)
__device__ unsigned long long g_tp_stamps[4096][10];
#define TP_STAMP(i)                                                                   \
    do {                                                                              \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                   \
        if (threadIdx.x == 0 && b < 4096) g_tp_stamps[b][i] = t_;                     \
    } while (0)
#else
#define TP_STAMP(i) ((void)0)
#endif

}  // namespace cmamd

#include "theorypass_body.h"

namespace cmamd {

// NB: the most 16-slot blocks any item uses.  With slot reuse the headline
// items need at most two, and four accumulators fit three waves per SIMD
// (168 VGPRs); NB = 4 keeps the general case at two.
template <int NB>
__global__ __launch_bounds__(256, NB <= 2 ? 3 : 2) void theory_window_kernel(TPDev c, const double *__restrict__ dl, long long ld_field,
                                                           long long ld_walker, int W, int tiles, int vec_ok)
{
    constexpr int LPL = 8, STEP = 4 * LPL, NSUB = TP_CHUNK / STEP, WROW = STEP + 2, NCB = TP_MAXCOL / 16;
    __shared__ __attribute__((aligned(16))) double wsh[2 * NCB * 16 * WROW];   // [buf][col block][col][l]
    __shared__ TPCol csh[TP_MAXCOL];      // the item's column descriptors
    __shared__ double xsh[TP_MAXCOL];     // and their data values (plik X)
    __shared__ unsigned long long esh[TP_MAXSTEP];            // slots ending at each step
    __shared__ unsigned char msh[TP_MAXSTEP * TP_MAXCOL];     // slot -> column at each step
    // the (item, walker tile) of this block comes from the host's plan (plan_units)
    const int b = blockIdx.x;
    const int2 unit = c.units[b];
    const int item = unit.x, tile = unit.y;
    (void)tiles;
    if (item < 0) return;
    TP_STAMP(0);
#ifdef CMAMD_STAMPS
    const unsigned long long rt0_ = __builtin_amdgcn_s_memrealtime();
#endif
    const TPItem it = c.items[item];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 15, kq = lane >> 4;
    const int w = tile * 64 + wave * 16 + li;
    const int wl = min(w, W - 1);
    const double *Df = dl + (long long)wl * ld_walker + (long long)it.field * ld_field;
    const int ncb = it.nsb;
    const int nstep = it.nst;
    double t[LPL], tn[LPL], tnn[LPL], a[LPL];
    auto load_t = [&](int st, double *dst) {
        const int lb = it.l0 + st * STEP + 2 * kq;
        if (vec_ok && it.l0 + st * STEP + STEP - 1 <= it.l1) {
#pragma unroll
            for (int q = 0; q < LPL / 2; q++) {
                const double2 v = *reinterpret_cast<const double2 *>(Df + lb + 8 * q);
                dst[2 * q] = v.x;
                dst[2 * q + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int q = 0; q < LPL / 2; q++)
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int l = lb + 8 * q + h;
                    dst[2 * q + h] = (l <= it.l1) ? Df[l] : 0.0;
                }
        }
    };
    // weights [nch][ncb][16][TP_CHUNK]; thread tid moves column tid/16, l 2 (tid%16) .. +1 of each block
    // (named registers, not arrays: a runtime block count would put an array in scratch)
    const int wc = tid >> 4, wp = 2 * (tid & 15);
    double2 wr0{}, wr1{}, wr2{}, wr3{};
    auto fetch_w = [&](int st) {
        const int ch = st / NSUB, sub = st % NSUB;
        const double *base = c.w + it.woff + (long long)ch * ncb * 16 * TP_CHUNK + sub * STEP + wc * TP_CHUNK + wp;
        const unsigned m = (unsigned)(it.act >> (4 * st)) & 15u;
        if (m & 1u) wr0 = *reinterpret_cast<const double2 *>(base);
        if (m & 2u) wr1 = *reinterpret_cast<const double2 *>(base + 16 * TP_CHUNK);
        if (m & 4u) wr2 = *reinterpret_cast<const double2 *>(base + 2 * 16 * TP_CHUNK);
        if (m & 8u) wr3 = *reinterpret_cast<const double2 *>(base + 3 * 16 * TP_CHUNK);
    };
    auto store_w = [&](int buf, int st) {
        double *d = wsh + (buf * NCB * 16 + wc) * WROW + wp;
        const unsigned m = (unsigned)(it.act >> (4 * st)) & 15u;
        if (m & 1u) *reinterpret_cast<double2 *>(d) = wr0;
        if (m & 2u) *reinterpret_cast<double2 *>(d + 16 * WROW) = wr1;
        if (m & 4u) *reinterpret_cast<double2 *>(d + 2 * 16 * WROW) = wr2;
        if (m & 8u) *reinterpret_cast<double2 *>(d + 3 * 16 * WROW) = wr3;
    };
    auto read_w = [&](int buf, int cb) {   // A operand: column li of block cb at the lane's LPL l
        const double *src = wsh + ((buf * NCB + cb) * 16 + li) * WROW + 2 * kq;
#pragma unroll
        for (int q = 0; q < LPL / 2; q++) {
            const double2 v = *reinterpret_cast<const double2 *>(src + 8 * q);
            a[2 * q] = v.x;
            a[2 * q + 1] = v.y;
        }
    };
    // two accumulators per block (even / odd MFMA steps), so consecutive MFMAs
    // of a block do not wait on each other; summed at the end
    f64x4 acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    f64x4 bcc0 = acc0, bcc1 = acc0, bcc2 = acc0, bcc3 = acc0;
    auto mfma_block = [&](int buf, int cb, f64x4 &acc, f64x4 &bcc) {
        read_w(buf, cb);
#pragma unroll
        for (int s = 0; s < LPL; s += 2) {
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], t[s], acc, 0, 0, 0);
            bcc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s + 1], t[s + 1], bcc, 0, 0, 0);
        }
    };
    // the theory rows run two steps ahead of the MFMAs, the weights one
    load_t(0, t);
    fetch_w(0);
    if (nstep > 1) load_t(1, tn);
    // epilogue operands, fetched behind the first step's loads: column
    // descriptors and X values into LDS, each stage's calibration per lane
    if (tid < it.ncol) {
        const TPCol d = c.cols[it.cdesc + tid];
        csh[tid] = d;
        const int kind = d.out ? c.out[1].kind : c.out[0].kind;
        const double *X = d.out ? c.out[1].X : c.out[0].X;
        xsh[tid] = kind == 1 ? X[d.row] : 0.0;
    }
    if (tid < nstep) esh[tid] = c.emit[it.soff + tid];
    for (int q = tid; q < nstep * (TP_MAXCOL / 4); q += 256)
        reinterpret_cast<unsigned int *>(msh)[q] =
            reinterpret_cast<const unsigned int *>(c.cmap + (long long)it.soff * TP_MAXCOL)[q];
    double c2[TP_MAXOUT], rc2[TP_MAXOUT];   // cal^2 and its reciprocal (div_rn)
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
    store_w(0, 0);
    __syncthreads();
    TP_STAMP(1);
    // D: walker = lane&15, slot = 16 cb + (lane>>4) + 4 r.  A column's sum is
    // written after the MFMAs of its last step, and its slot is zeroed for the
    // next column: the sum is the same MFMA chain as with a slot of its own
    // (the steps outside its range only ever added products with zero weight)
    auto emit = [&](int st, unsigned long long e, int cb, f64x4 &acc, f64x4 &bcc) {
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int slot = 16 * cb + kq + 4 * r;
            if (!((e >> slot) & 1ull)) continue;
            const int col = msh[st * TP_MAXCOL + slot];
            double v = acc[r] + bcc[r];
            acc[r] = 0.0;
            bcc[r] = 0.0;
            if (w >= W) continue;
            const TPCol d = csh[col];
            const bool o1 = d.out != 0;   // selects, not a dynamically indexed kernel argument
            const int kind = o1 ? c.out[1].kind : c.out[0].kind;
            double *out = o1 ? c.out[1].out : c.out[0].out;
            if (d.cal) v = div_rn(v, o1 ? c2[1] : c2[0], o1 ? rc2[1] : rc2[0]);   // = v / cal^2
            if (kind == 0) {
                out[(long long)d.row * W + w] = v;
            } else {
                const int ld = o1 ? c.out[1].ld : c.out[0].ld;
                out[(long long)w * ld + d.row] = xsh[col] - v;
            }
        }
    };
    for (int st = 0; st < nstep; st++) {
        const bool more = st + 1 < nstep;
        const int cur = st & 1;
        if (more) fetch_w(st + 1);                     // in flight across this step's MFMAs
        if (st + 2 < nstep) load_t(st + 2, tnn);
        const unsigned m = (unsigned)(it.act >> (4 * st)) & 15u;   // blocks with weight in this step
        if (m & 1u) mfma_block(cur, 0, acc0, bcc0);
        if (m & 2u) mfma_block(cur, 1, acc1, bcc1);
        if constexpr (NB > 2) {
            if (m & 4u) mfma_block(cur, 2, acc2, bcc2);
            if (m & 8u) mfma_block(cur, 3, acc3, bcc3);
        }
        const unsigned long long e = esh[st];
        if (e & 0xffffull) emit(st, e, 0, acc0, bcc0);
        if (e & 0xffff0000ull) emit(st, e, 1, acc1, bcc1);
        if constexpr (NB > 2) {
            if (e & 0xffff00000000ull) emit(st, e, 2, acc2, bcc2);
            if (e & 0xffff000000000000ull) emit(st, e, 3, acc3, bcc3);
        }
        if (more) {
            store_w(cur ^ 1, st + 1);      // buffer cur ^ 1 was last read before the previous barrier
            __syncthreads();
#pragma unroll
            for (int s = 0; s < LPL; s++) {
                t[s] = tn[s];
                tn[s] = tnn[s];
            }
        }
    }
    TP_STAMP(2);
#ifdef CMAMD_STAMPS
    if (threadIdx.x == 0 && b < 4096) {
        g_tp_stamps[b][4] = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        g_tp_stamps[b][5] = __builtin_amdgcn_s_getreg((3 << 11) | 20);
        g_tp_stamps[b][6] = item;
        g_tp_stamps[b][7] = (unsigned long long)nstep * 1000 + __builtin_popcountll(it.act);
    }
#endif
    TP_STAMP(3);
#ifdef CMAMD_STAMPS
    const unsigned long long rt1_ = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && b < 4096) {
        g_tp_stamps[b][8] = rt0_;
        g_tp_stamps[b][9] = rt1_;
    }
#endif
}

// The vectorised pass (theorypass_body.h) as a kernel of its own
template <int NB>
__global__ __launch_bounds__(256, NB <= 2 ? 3 : 2) void theory_window_vec(TPDev c, const double *__restrict__ dl,
                                                                         long long ld_field, long long ld_walker, int W)
{
    __shared__ __attribute__((aligned(16))) char lds[tp_vec_lds_bytes<NB>()];
    tp_vec_body<NB, false, true>(c, dl, ld_field, ld_walker, W, lds, blockIdx.x);
}

// The pass over two theory sets in one launch (the dragging steps' end and
// start points): blocks [0, n) run set a's table, [n, 2n) set b's; the first
// block of each also zeroes that set's quadratic-form tickets (zero[k], nz[k]
// words) for the in-launch-combined quadratic form that follows.
__global__ __launch_bounds__(256, 3) void theory_window_pair(TPDev ca, const double *__restrict__ dla, long long lfa,
                                                             long long lwa, TPDev cb, const double *__restrict__ dlb,
                                                             long long lfb, long long lwb, int W, int n,
                                                             unsigned int *za, unsigned int *zb, int nz)
{
    __shared__ __attribute__((aligned(16))) char lds[tp_vec_lds_bytes<2>()];
    const bool second = (int)blockIdx.x >= n;
    const int b = (int)blockIdx.x - (second ? n : 0);
    if (b == 0 && (int)threadIdx.x < nz) (second ? zb : za)[threadIdx.x] = 0u;
    if (second)
        tp_vec_body<2, false, true>(cb, dlb, lfb, lwb, W, lds, b);
    else
        tp_vec_body<2, false, true>(ca, dla, lfa, lwa, W, lds, b);
}

// ------------------------------------------------------------------ host side

bool TheoryPass::build(const std::vector<WinStage> &stages) {
    if (stages.empty() || stages.size() > (size_t)TP_MAXOUT) return false;
    struct C { int lo, hi, stage, col; };
    std::map<int, std::vector<C>> byf;
    for (size_t s = 0; s < stages.size(); s++)
        for (size_t k = 0; k < stages[s].cols.size(); k++) {
            const WinCol &wc = stages[s].cols[k];
            if (wc.hi < wc.lo || wc.lo < 0) return false;
            byf[wc.field].push_back(C{wc.lo, wc.hi, (int)s, (int)k});
        }
    max_nsb = 0;
    std::vector<TPItem> its;
    std::vector<TPCol> cols;
    std::vector<double> w;
    std::vector<unsigned long long> emit;
    std::vector<unsigned char> cmap;
    for (auto &kv : byf) {
        auto &v = kv.second;
        // by start, the longest first among equal starts: a long column that
        // opens a new range then starts the new item before the short ones
        // sharing its start are considered for the previous one
        std::stable_sort(v.begin(), v.end(),
                         [](const C &x, const C &y) { return x.lo < y.lo || (x.lo == y.lo && x.hi > y.hi); });
        std::vector<std::vector<C>> groups;
        std::vector<C> cur;
        int a = 0, bnd = -1;
        for (const C &x : v) {
            // a column that overlaps the group joins it; otherwise it starts a
            // new group once the group would pass TP_MAXL l or TP_MAXCOL columns
            if (!cur.empty() && x.lo > bnd &&
                (std::max(bnd, x.hi) - a + 1 > TP_MAXL || (int)cur.size() + 1 > TP_MAXCOL)) {
                groups.push_back(cur);
                cur.clear();
            }
            if (cur.empty()) {
                a = x.lo;
                bnd = x.hi;
            } else {
                bnd = std::max(bnd, x.hi);
            }
            cur.push_back(x);
            if ((int)cur.size() > TP_MAXCOL) {
                fprintf(stderr, "theorypass: field %d [%d, %d] needs %zu columns\n", kv.first, a, bnd, cur.size());
                return false;
            }
        }
        if (!cur.empty()) groups.push_back(cur);
        for (auto &g : groups) {
            // columns: the wide ones (CMBlikes windows, every step) first, then by start,
            // so the narrow ones (plik bins) of one block are active in few steps
            std::stable_sort(g.begin(), g.end(), [](const C &x, const C &y) {
                const int wx = x.hi - x.lo, wy = y.hi - y.lo;
                if ((wx >= TP_CHUNK) != (wy >= TP_CHUNK)) return wx >= TP_CHUNK;
                return x.lo < y.lo;
            });
            TPItem it{};
            it.field = kv.first;
            int lo = g[0].lo, hi = g[0].hi;
            for (auto &x : g) {
                lo = std::min(lo, x.lo);
                hi = std::max(hi, x.hi);
            }
            it.l0 = lo & ~1;                      // even: 16-byte theory loads
            it.l1 = hi;
            it.nch = (it.l1 - it.l0 + TP_CHUNK) / TP_CHUNK;
            it.nst = (it.l1 - it.l0 + 32) / 32;
            if (it.nst > TP_MAXSTEP || (int)g.size() > TP_MAXCOL) {
                fprintf(stderr, "theorypass: field %d [%d, %d] longer than %d l\n", kv.first, it.l0, it.l1,
                        TP_MAXSTEP * 32);
                return false;
            }
            it.ncol = (int)g.size();
            it.cdesc = (int)cols.size();
            it.woff = (long long)w.size();
            const int nstep = it.nst;
            // steps of each column, and its slot: the lowest slot whose previous
            // column ended before this one's first step (g: wide ones first, then by l)
            std::vector<int> s0(g.size()), s1(g.size()), slot(g.size());
            std::vector<int> slot_end;                    // last step of the slot's current column
            for (size_t q = 0; q < g.size(); q++) {
                const WinCol &wc = stages[g[q].stage].cols[g[q].col];
                s0[q] = std::max(0, (wc.lo - it.l0) / 32);
                s1[q] = std::min(nstep - 1, (wc.hi - it.l0) / 32);
                int k = 0;
                while (k < (int)slot_end.size() && slot_end[k] >= s0[q]) k++;
                if (k == (int)slot_end.size()) slot_end.push_back(0);
                slot_end[k] = s1[q];
                slot[q] = k;
            }
            it.nsb = ((int)slot_end.size() + 15) / 16;
            max_nsb = std::max(max_nsb, it.nsb);
            it.soff = (int)emit.size();
            // slot -> column per step (255: none), and the slots whose column ends at each step
            std::vector<unsigned char> sm((size_t)nstep * TP_MAXCOL, 255);
            std::vector<unsigned long long> em(nstep, 0ull);
            for (size_t q = 0; q < g.size(); q++) {
                for (int st = s0[q]; st <= s1[q]; st++) {
                    sm[(size_t)st * TP_MAXCOL + slot[q]] = (unsigned char)q;
                    it.act |= 1ull << (4 * st + slot[q] / 16);
                }
                em[s1[q]] |= 1ull << slot[q];
            }
            for (int ch = 0; ch < it.nch; ch++)
                for (int cb = 0; cb < it.nsb; cb++)
                    for (int sl = 16 * cb; sl < 16 * cb + 16; sl++)
                        for (int k = 0; k < TP_CHUNK; k++) {
                            const int l = it.l0 + ch * TP_CHUNK + k;
                            const int stk = (ch * TP_CHUNK + k) / 32;   // steps past nstep: padding
                            const int q = stk < nstep ? sm[(size_t)stk * TP_MAXCOL + sl] : 255;
                            double x = 0.0;
                            if (q != 255) {
                                const WinCol &wc = stages[g[q].stage].cols[g[q].col];
                                if (l >= wc.lo && l <= wc.hi) x = wc.w[l - wc.lo];
                            }
                            w.push_back(x);
                        }
            for (size_t q = 0; q < g.size(); q++) {
                const WinCol &wc = stages[g[q].stage].cols[g[q].col];
                cols.push_back(TPCol{g[q].stage, wc.row, wc.cal, 0});
            }
            emit.insert(emit.end(), em.begin(), em.end());
            cmap.insert(cmap.end(), sm.begin(), sm.end());
            its.push_back(it);
        }
    }
    items = its;
    nstage = (int)stages.size();
    auto up = [](DevBuf &d, const void *p, size_t bytes) {
        d.alloc(std::max<size_t>(16, bytes));
        if (bytes) d.upload(p, bytes);
    };
    up(d_items, items.data(), items.size() * sizeof(TPItem));
    up(d_cols, cols.data(), cols.size() * sizeof(TPCol));
    w.resize(w.size() + 4 * 16 * TP_CHUNK, 0.0);   // theory_window_vec reads four blocks of every item
    up(d_w, w.data(), w.size() * 8);
    up(d_emit, emit.data(), emit.size() * sizeof(unsigned long long));
    up(d_cmap, cmap.data(), cmap.size());
    return true;
}

// Block table.  The blocks are dealt to the XCDs round-robin (block b on XCD
// b % 8), and within an XCD the measured dispatch puts its j-th block on CU
// j % (CUs per XCD) while every block fits at once (block stamps,
// tools/tp_stamps.py).  With walker tiles of an item on consecutive blocks,
// the CUs that received a third block got two long items (TT / TE ranges with
// lensing and plik columns: two MFMA blocks per step) and set the kernel's end
// at 27.8 us against a median CU end of 22.8 us.  So the units (item, tile) are
// placed by cost instead: the items go to XCDs by longest-processing-time over
// their summed cost (all tiles of an item on one XCD: its weights in one L2),
// then each XCD's units to its CUs the same way, and the table lists them round
// by round (CU c's k-th unit at j = k * ncu + c); a CU with fewer units has an
// empty entry there.  Cost of a unit: its active 16-column MFMA block-steps +
// 1.1 per 32-l step (a CU's end time, fitted over the 256 CUs' stamps, was
// 16.1 us + 148 ns per block-step + 166 ns per step; no per-block term).  The
// kernel went from 27.7 to 26.2 us (CU ends 22.4-25.4 us instead of
// 18-27.8).  Every unit appears once, so the outputs do not depend on the plan.
void TheoryPass::plan_units(int tiles) {
    int dev = 0, ncu = 256;
    HIP_CHECK(hipGetDevice(&dev));
    HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int NX = 8, cpx = std::max(1, ncu / NX);
    const int ni = (int)items.size();
    std::vector<double> cost(ni);
    for (int i = 0; i < ni; i++)
        cost[i] = __builtin_popcountll(items[i].act) + 1.1 * items[i].nst;
    std::vector<int> ord(ni);
    for (int i = 0; i < ni; i++) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return cost[a] > cost[b]; });
    std::vector<double> xload(NX, 0.0);
    std::vector<std::vector<int>> xitems(NX);
    for (int i : ord) {
        const int x = (int)(std::min_element(xload.begin(), xload.end()) - xload.begin());
        xload[x] += cost[i] * tiles;
        xitems[x].push_back(i);
    }
    // per XCD, per CU: its units in placement order
    std::vector<std::vector<std::vector<int2>>> cu(NX, std::vector<std::vector<int2>>(cpx));
    int rounds = 0;
    for (int x = 0; x < NX; x++) {
        std::vector<double> load(cpx, 0.0);
        for (int i : xitems[x])          // already by cost, descending
            for (int t = 0; t < tiles; t++) {
                const int k = (int)(std::min_element(load.begin(), load.end()) - load.begin());
                load[k] += cost[i];
                cu[x][k].push_back(int2{i, t});
                rounds = std::max(rounds, (int)cu[x][k].size());
            }
    }
    std::vector<int2> table((size_t)NX * cpx * rounds, int2{-1, 0});
    for (int x = 0; x < NX; x++)
        for (int k = 0; k < cpx; k++)
            for (size_t r = 0; r < cu[x][k].size(); r++) table[((size_t)r * cpx + k) * NX + x] = cu[x][k][r];
    nblk = (int)table.size();
    per_round = NX * cpx;
    d_units.alloc(table.size() * sizeof(int2));
    d_units.upload(table.data(), table.size() * sizeof(int2));
    unit_tiles = tiles;
}

void TheoryPass::launch_pair(const double *dla, long long lfa, long long lwa, const TPOut *oa, unsigned int *za,
                             const double *dlb, long long lfb, long long lwb, const TPOut *ob, unsigned int *zb,
                             int nz, int W, hipStream_t stream) {
    if (W <= 0 || items.empty()) return;
    if (!vec_ok(dla, lfa, lwa) || (dlb && !vec_ok(dlb, lfb, lwb)) || nz > 256) fail(CMBL_ERR_ARG, "internal: pass pair");
    const TPDev ca = dev_args(oa, W), cb = dlb ? dev_args(ob, W) : ca;
    timed_launch("theory_window_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
        hipExtLaunchKernelGGL(theory_window_pair, dim3(dlb ? 2 * nblk : nblk), dim3(256), 0, stream, e0, e1, 0, ca, dla,
                              lfa, lwa, cb, dlb, lfb, lwb, W, nblk, za, zb, nz);
    });
    HIP_CHECK(hipGetLastError());
}

bool TheoryPass::vec_ok(const double *dl, long long ld_field, long long ld_walker) const {
    // (four blocks would not fit the registers: theory_window_kernel<4>)
    return ((reinterpret_cast<uintptr_t>(dl) & 15) == 0) && ld_field % 2 == 0 && ld_walker % 2 == 0 && max_nsb <= 2;
}

TPDev TheoryPass::dev_args(const TPOut *outs, int W) {
    TPDev c{};
    c.items = d_items.as<TPItem>();
    c.cols = d_cols.as<TPCol>();
    c.w = d_w.as<double>();
    c.emit = d_emit.as<unsigned long long>();
    c.cmap = d_cmap.as<unsigned char>();
    c.nitem = (int)items.size();
    for (int s = 0; s < nstage; s++) c.out[s] = outs[s];
    const int tiles = (W + 63) / 64;
    if (tiles != unit_tiles) plan_units(tiles);
    c.units = d_units.as<int2>();
    c.nblk = nblk;
    return c;
}

void TheoryPass::launch(const double *dl, long long ld_field, long long ld_walker, const TPOut *outs, int W,
                        hipStream_t stream) {
    if (W <= 0 || items.empty()) return;
    const TPDev c = dev_args(outs, W);
    const int vec_ok = ((reinterpret_cast<uintptr_t>(dl) & 15) == 0) && ld_field % 2 == 0 && ld_walker % 2 == 0;
    const int tiles = (W + 63) / 64;
    if (this->vec_ok(dl, ld_field, ld_walker)) {
        timed_launch("theory_window_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
            hipExtLaunchKernelGGL(theory_window_vec<2>, dim3(nblk), dim3(256), 0, stream, e0, e1, 0, c, dl, ld_field,
                                  ld_walker, W);
        });
        HIP_CHECK(hipGetLastError());
        return;
    }
    timed_launch("theory_window_kernel", stream, [&](hipEvent_t e0, hipEvent_t e1) {
        if (max_nsb <= 2)
            hipExtLaunchKernelGGL(theory_window_kernel<2>, dim3(nblk), dim3(256), 0, stream, e0, e1, 0, c, dl,
                                  ld_field, ld_walker, W, tiles, vec_ok);
        else
            hipExtLaunchKernelGGL(theory_window_kernel<4>, dim3(nblk), dim3(256), 0, stream, e0, e1, 0, c, dl,
                                  ld_field, ld_walker, W, tiles, vec_ok);
    });
    HIP_CHECK(hipGetLastError());
}

}  // namespace cmamd

#ifdef CMAMD_STAMPS
extern "C" int cmamd_debug_tp_stamps(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(cmamd::g_tp_stamps), sizeof(cmamd::g_tp_stamps)) == hipSuccess ? 0 : -5;
}
#endif
