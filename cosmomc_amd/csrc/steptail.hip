// The unified step launch's workgroup rows (see steptail.h).
#include <cstdlib>
#include <string>
#include <vector>

#include "steptail.h"

namespace cmamd {

// The rows' order: CMAMD_TAIL_ORDER lists the roles (q: quadratic form, g:
// chi^2, p: pass) in dispatch order; "q*p" deals the q and p rows in
// proportion to their counts, interleaved.  Default "gqp", "mqp" with the chi^2 folded ("qpg" measured 58.4
// against 40.9 us/step, round 4; with the Metropolis rows placed earlier, 61-94
// against 38.5, round 5: profiles/r05_schedules.txt).
std::vector<int2> tail_rows(int nq, int ng, int np, int nm) {
    static const char *env = std::getenv("CMAMD_TAIL_ORDER");
    // with the chi^2 folded into the Metropolis workgroups (ng = 0) they come first and
    // compute it while the quadratic form runs: "mqp" 32.6-32.7 against "gqp" 41.0 and
    // the chi^2 as rows of its own 33.6-33.8 us a middle launch (round 6, r6a)
    const std::string order = env && *env ? env : (ng > 0 ? "gqp" : "mqp");
    const int cnt[3] = {(nq + 7) / 8, (ng + 7) / 8, (np + 7) / 8};
    auto role = [](char c) { return c == 'q' ? TAIL_QF : c == 'g' ? TAIL_GAUSS : c == 'p' ? TAIL_PASS : -1; };
    std::vector<int2> rows;
    int done[3] = {0, 0, 0};
    auto emit = [&](int r) { rows.push_back(int2{r, done[r]++}); };
    bool mh_done = false;
    auto emit_mh = [&]() {
        for (int k = 0; k < (nm + 7) / 8; k++) rows.push_back(int2{TAIL_MH, k});
        mh_done = true;
    };
    for (size_t i = 0; i < order.size(); i++) {
        if (order[i] == 'm' && !mh_done) {   // the Metropolis rows here: they then wait resident for
            emit_mh();                       // their tiles' producers (64 of the launch's >= 512 slots)
            continue;
        }
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
    // the Metropolis rows last unless the order places them ('m'): they wait
    // for their tile's quadratic-form and chi^2 workgroups
    if (!mh_done) emit_mh();
    return rows;
}

}  // namespace cmamd

