// The step tail of the split pipelined fast steps (see steptail.h).
#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "qfs_body.h"
#include "smallgauss.h"
#include "steptail.h"
#include "theorypass_body.h"

namespace cmamd {

#ifdef CMAMD_STAMPS
// step_tail_kernel with all three roles (tools/uni_stamps.py): start, -, XCC id, end, role + 1
__device__ unsigned long long g_tail_stamps[2048][5];
#endif

// Roles by rows of 8 workgroups (tail_rows, steptail.h).

__global__ __launch_bounds__(256, 3) void step_tail_kernel(StepTail t, const int2 *__restrict__ rows)
{
    extern __shared__ __attribute__((aligned(16))) double tail_lds[];
    const int2 rr = rows[blockIdx.x >> 3];
    const int lb = rr.y * 8 + (blockIdx.x & 7);
#ifdef CMAMD_STAMPS
    const bool stamp = t.nq && t.np && threadIdx.x == 0 && blockIdx.x < 2048;
    if (stamp) {
        unsigned xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        g_tail_stamps[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
        g_tail_stamps[blockIdx.x][2] = xcc & 15;
        g_tail_stamps[blockIdx.x][4] = 0;
    }
    struct End {
        bool on;
        int role;
        __device__ ~End() {
            if (on) {
                g_tail_stamps[blockIdx.x][3] = __builtin_amdgcn_s_memrealtime();
                g_tail_stamps[blockIdx.x][4] = role + 1;
            }
        }
    } end_{stamp, rr.x};
#endif
    if (rr.x == TAIL_QF) {
        if (lb >= t.nq) return;
        int item_ix, tile;
        qf_place(lb, t.q.src.n_items, t.q.src.xcd_map, item_ix, tile);
        qfs_body(tail_lds, item_ix, tile, t.q);
    } else if (rr.x == TAIL_GAUSS) {
        if (lb < t.ng) small_gauss_body<SMALL_WT, true>(t.g, tail_lds, lb);
    } else if (rr.x == TAIL_PASS) {
        if (lb >= t.np) return;
        tp_vec_body<2, false, true>(t.tp, t.dl, t.ld_field, t.ld_walker, t.W, reinterpret_cast<char *>(tail_lds), lb);
    }
}

// ------------------------------------------------------------------ host side

// The rows' order: CMAMD_TAIL_ORDER lists the roles (q: quadratic form, g:
// chi^2, p: pass) in dispatch order; "q*p" deals the q and p rows in
// proportion to their counts, interleaved.  Default "qpg" for the step tails
// and "gqp" for the unified launch (nm > 0; "qpg" measured 58.4 against 40.9
// us/step there).
std::vector<int2> tail_rows(int nq, int ng, int np, int nm) {
    static const char *env = std::getenv("CMAMD_TAIL_ORDER");
    const std::string order = env && *env ? env : (nm > 0 ? "gqp" : "qpg");
    const int cnt[3] = {(nq + 7) / 8, (ng + 7) / 8, (np + 7) / 8};
    auto role = [](char c) { return c == 'q' ? TAIL_QF : c == 'g' ? TAIL_GAUSS : c == 'p' ? TAIL_PASS : -1; };
    std::vector<int2> rows;
    int done[3] = {0, 0, 0};
    auto emit = [&](int r) { rows.push_back(int2{r, done[r]++}); };
    for (size_t i = 0; i < order.size(); i++) {
        const int r = role(order[i]);
        if (r < 0) continue;
        if (i + 2 < order.size() && order[i + 1] == '*' && role(order[i + 2]) >= 0) {
            const int s = role(order[i + 2]);
            const int a = cnt[r] - done[r], b = cnt[s] - done[s];
            for (int k = 0, ka = 0; k < a + b; k++) {   // r's rows spread evenly over the a + b
                if ((long long)(k + 1) * a / (a + b) > ka) {
                    emit(r);
                    ka++;
                } else {
                    emit(s);
                }
            }
            i += 2;
            continue;
        }
        while (done[r] < cnt[r]) emit(r);
    }
    for (int r = 0; r < 3; r++)   // roles the order left out
        while (done[r] < cnt[r]) emit(r);
    // the Metropolis rows last, whatever the order: they wait for their tile's
    // quadratic-form and chi^2 workgroups, which are then all dispatched first
    for (int k = 0; k < (nm + 7) / 8; k++) rows.push_back(int2{TAIL_MH, k});
    return rows;
}

size_t step_tail_lds_bytes() {
    size_t b = (size_t)QFS_LDS_DOUBLES * 8;
    b = std::max(b, (size_t)tp_vec_lds_bytes<2, false>());
    b = std::max(b, (size_t)small_gauss_lds_doubles<SMALL_WT>(SMALL_NX) * 8);
    return b;
}

void launch_step_tail(const StepTail &t, StepTailPlan &plan, hipStream_t stream, const char *prof_name) {
    if (t.nq + t.ng + t.np == 0) return;
    if (t.nq && (t.q.src.n_items <= 0 || !t.q.S)) fail(CMBL_ERR_ARG, "internal: step tail without its operands");
    if (plan.key[0] != t.nq || plan.key[1] != t.ng || plan.key[2] != t.np) {
        const std::vector<int2> rows = tail_rows(t.nq, t.ng, t.np, 0);
        plan.d_rows.alloc(rows.size() * sizeof(int2));
        plan.d_rows.upload(rows.data(), rows.size() * sizeof(int2));
        plan.nrows = (int)rows.size();
        plan.key[0] = t.nq;
        plan.key[1] = t.ng;
        plan.key[2] = t.np;
    }
    size_t lds = 0;
    if (t.nq) lds = std::max(lds, (size_t)QFS_LDS_DOUBLES * 8);
    if (t.np) lds = std::max(lds, (size_t)tp_vec_lds_bytes<2, false>());
    if (t.ng) lds = std::max(lds, (size_t)small_gauss_lds_doubles<SMALL_WT>(t.g.d.nX) * 8);
    const dim3 grid((unsigned)plan.nrows * 8);
    const int2 *rows = plan.d_rows.as<int2>();
    timed_launch(prof_name, stream, [&](hipEvent_t e0, hipEvent_t e1) {
        hipExtLaunchKernelGGL(step_tail_kernel, grid, dim3(256), lds, stream, e0, e1, 0, t, rows);
    });
    HIP_CHECK(hipGetLastError());
}

}  // namespace cmamd

#ifdef CMAMD_STAMPS
extern "C" int cmamd_debug_tail_stamps(unsigned long long *host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(cmamd::g_tail_stamps), sizeof(cmamd::g_tail_stamps)) == hipSuccess ? 0
                                                                                                                 : -5;
}
#endif
