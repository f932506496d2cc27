// xsched_sim.cpp -- CPU check that every rank of a job issues the same records all-reduces
// (tk_xsched.h), whatever its rank-local state.
//
// The REAL native driver (tk_solver_run, csrc/tk_solver.cpp) and host math (tk_host.cpp)
// run against a stand-in of the decomposition's exchange bookkeeping that follows
// tk_abi.cpp call for call (tk_decomp_init / step / sweep / flush / records / basis_mul:
// local record completion, the deferred bookkeeping of one-sweep kernels, need_slots,
// XSched), with the RCCL call replaced by a log line (first slot, last slot, element count).
// Every simulated job runs its ranks one after another; tk_decomp_agree returns the
// element-wise max of what all ranks of the job submit (as the all-reduce would).
//
// Rank kinds:  ONESWEEP  one-sweep Arnoldi/Lanczos (step j's record is written by step j+1's
//                        launch or an explicit bookkeeping flush)
//              CGS2      two-sweep / TTR kernels (step j's record written by step j itself)
//              EMPTY     a rank holding no factor (nf = 0), kernels skipped: as CGS2
// Output: one line per job, "JOB <name> ranks=<n> identical=<0|1> calls=<n> first=<log>".
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <ctype.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>

#include "../../include/tk.h"
#include "../../tensorkrylov.jl_amd/csrc/tk_xsched.h"

using tk::XSched;

static char g_err[512];
tk_status tk_fail_internal(int code, const char* msg) {   // (C++ linkage, as tk_abi.cpp)
    snprintf(g_err, sizeof g_err, "%s", msg);
    return code;
}
extern "C" const char* tk_last_error(void) { return g_err; }
extern "C" int tk_record_len(int kmax) { return 2 * kmax + 10; }

enum Kind { ONESWEEP = 0, CGS2 = 1, EMPTY = 2 };

struct tk_decomp {
    int kind, kmax, d, m;
    int jnext = 0, bk_j = -1;
    bool pending = false;
    XSched xs;
    std::vector<std::string> log;
    int agree_idx = 0;
};

// the job's agreement: every rank's submissions (tk_solver_run's: worker count, depth, the
// evaluation-split flag and its negation), max taken when a rank asks
static std::vector<std::vector<int>> g_sub;   // [rank][value]
static std::vector<int> g_group;              // [rank] TKHIP_XCH_GROUP
static int g_rank = 0;
// XSCHED_SIM_LOCAL=1 (negative control): no agreement -- each rank keeps its own worker
// count, depth and group size, as before tk_decomp_agree / the create preflight existed
static bool g_local = false;

static void xsend(tk_decomp* dc, XSched::Range r) {
    if (r.first > r.second) return;
    for (int s = r.first; s <= r.second; ++s)
        if (!dc->xs.written(s)) {
            fprintf(stderr, "rank %d: slot %d exchanged before it is written\n", g_rank, s);
            exit(3);
        }
    char b[96];
    snprintf(b, sizeof b, "[%d,%d]x%d", r.first, r.second, (r.second - r.first + 1) * dc->d * dc->m);
    dc->log.push_back(b);
}
static void xsend_single(tk_decomp* dc, int slot) {
    char b[96];
    snprintf(b, sizeof b, "[%d,%d]x%d", slot, slot, dc->d * dc->m);
    dc->log.push_back(b);
}
static void bk_flush(tk_decomp* dc) {
    if (dc->bk_j < 0) return;
    dc->xs.complete(dc->bk_j + 1);
    dc->bk_j = -1;
}
static void need_slots(tk_decomp* dc, int S) {
    if (S <= dc->xs.sent) return;
    if (dc->bk_j >= 0 && dc->bk_j + 1 <= S) bk_flush(dc);
    xsend(dc, dc->xs.need(S));
}

extern "C" {

tk_status tk_decomp_agree(tk_decomp* dc, int* vals, int count) {
    // ranks run one after another: the values every rank submits are known up front
    (void)dc;
    if (g_local) return TK_OK;
    for (int i = 0; i < count; ++i) {
        int mx = vals[i];
        for (const auto& r : g_sub) mx = std::max(mx, r[i]);
        vals[i] = mx;
    }
    return TK_OK;
}

tk_status tk_decomp_init(tk_decomp* dc, double* rec_out) {
    (void)rec_out;
    bk_flush(dc);
    dc->jnext = 0;
    dc->pending = false;
    dc->xs.reset();
    dc->xs.complete(0);
    xsend(dc, dc->xs.need(0));
    return TK_OK;
}

tk_status tk_decomp_step(tk_decomp* dc, int j, double* rec_out) {
    if (j != dc->jnext || j >= dc->kmax) return tk_fail_internal(TK_ERR_STATE, "step out of order");
    if (dc->kind == ONESWEEP) {
        // the launch carries step j-1's bookkeeping; step j's is deferred
        if (dc->bk_j >= 0 && dc->bk_j != j - 1) bk_flush(dc);
        const int prev = dc->bk_j;
        dc->bk_j = j;
        if (prev == j - 1 && prev >= 0) dc->xs.complete(prev + 1);
        if (rec_out) bk_flush(dc);
    } else {
        dc->xs.complete(j + 1);
    }
    dc->pending = true;
    dc->jnext = j + 1;
    for (const XSched::Range& r : dc->xs.step_done(j)) xsend(dc, r);
    if (rec_out) need_slots(dc, j + 1);
    if (rec_out) memset(rec_out, 0, sizeof(double) * dc->d * dc->m);
    return TK_OK;
}

tk_status tk_decomp_gram_ahead(tk_decomp* dc, int* k_out) {   // (no collective: nothing to log)
    (void)dc;
    *k_out = 0;
    return TK_OK;
}
tk_status tk_decomp_gram(tk_decomp* dc, int f, int k, double* G) {   // (never reached: no Gram ahead)
    (void)dc;
    (void)f;
    (void)k;
    (void)G;
    return TK_ERR_STATE;
}

tk_status tk_decomp_records(tk_decomp* dc, int s0, int s1, double* out) {
    if (s1 > s0) need_slots(dc, std::min(s1 - 1, dc->jnext));
    memset(out, 0, sizeof(double) * (s1 - s0) * dc->d * dc->m);
    return TK_OK;
}

}  // extern "C"

static void flush(tk_decomp* dc) {
    bk_flush(dc);
    need_slots(dc, dc->jnext);
    if (dc->pending) {
        dc->pending = false;
        xsend_single(dc, dc->kmax + 1);
    }
}

struct RankCfg {
    int kind, threads, depth, group;
    int split = 0;   // 1: tk_solver_share over the job's ranks (threads, real mailbox)
};
static std::string g_key;   // the job's mailbox key

// one rank's whole call sequence: the Python driver's init + step 0 (records out), the
// native loop, then basis_mul / flush on convergence (tkamd/solver.py)
static std::vector<std::string> run_rank(const RankCfg& rc, int kmax, int d, double tol, int myrank, int nranks) {
    tk_decomp dc;
    dc.kind = rc.kind;
    dc.kmax = kmax;
    dc.d = d;
    dc.m = tk_record_len(kmax);
    dc.xs.group = rc.group;
    // tk_decomp_create's preflight: the group size is the max over the ranks
    if (!g_local)
        for (int g : g_group) dc.xs.group = std::max(dc.xs.group, g);
    std::vector<double> rec((size_t)d * dc.m);
    tk_decomp_init(&dc, rec.data());
    tk_decomp_step(&dc, 0, rec.data());
    std::vector<double> lmin(kmax, 1.0), al(kmax, 1.0), om(kmax, 1.0);
    std::vector<int> rank(kmax, 1);
    tk_solver* sv = nullptr;
    if (tk_solver_create(TK_ARNOLDI, d, kmax, 1, 1.0, lmin.data(), rank.data(), al.data(), om.data(), &sv)) {
        fprintf(stderr, "tk_solver_create: %s\n", g_err);
        exit(2);
    }
    if (rc.split == 1 && tk_solver_share(sv, g_key.c_str(), nranks, myrank)) {
        fprintf(stderr, "tk_solver_share: %s\n", g_err);
        exit(2);
    }
    // split = 2: this rank alone has a results source (an emulation table); the run's
    // agreement must then turn the split off on every rank
    std::vector<double> table((size_t)kmax * 6, 0.0);
    if (rc.split == 2 && tk_solver_share_emulated(sv, nranks, myrank, table.data())) {
        fprintf(stderr, "tk_solver_share_emulated: %s\n", g_err);
        exit(2);
    }
    std::vector<double> relres(kmax), proj(kmax), orth(kmax);
    int k_end = 0, outcome = 0;
    tk_status st = tk_solver_run(sv, &dc, tol, 2, rc.depth, rc.threads, relres.data(), proj.data(), orth.data(),
                                 &k_end, &outcome);
    if (st) {
        fprintf(stderr, "tk_solver_run: %d %s\n", st, g_err);
        exit(2);
    }
    char rb[96];
    snprintf(rb, sizeof rb, "relres[%d]=%.17g", k_end - 1, relres[k_end - 1]);
    std::vector<double> lam(1), Y((size_t)d * k_end);
    if (outcome == 1 && tk_solver_solution(sv, k_end, lam.data(), Y.data())) {   // (every rank: its y)
        fprintf(stderr, "rank %d: tk_solver_solution: %s\n", myrank, g_err);
        exit(5);
    }
    tk_solver_destroy(sv);
    if (outcome == 1) flush(&dc);   // basis_mul's flush of the pending column
    // the deferred orthogonality Gram (tkamd.solver._fill_deferred_orthogonality):
    // every rank flushes when the Gram of k_end columns reads the pending column -- decided
    // from the step sequence alone (columns < last_j are written on every path, column last_j
    // unless it waits in the one-sweep column buffer: even last_j) -- then the rank owning
    // factor 1 runs the Gram, which must start no collective: tk_decomp_gram refuses a Gram
    // that reads a pending column on a multi-rank handle
    const int last_j = dc.jnext - 1;
    if (k_end - 1 >= last_j + (last_j % 2 == 0 ? 0 : 1)) flush(&dc);
    const bool in_e = dc.kind == ONESWEEP && last_j % 2 == 0;
    if (dc.pending && k_end - 1 >= last_j + (in_e ? 0 : 1)) {
        fprintf(stderr, "rank %d: Gram with column %d pending\n", g_rank, dc.jnext);
        exit(4);
    }
    char b[64];
    snprintf(b, sizeof b, "end k=%d outcome=%d", k_end, outcome);
    dc.log.push_back(b);
    dc.log.push_back(rb);
    return dc.log;
}

static int run_job(const char* name, const std::vector<RankCfg>& ranks, int kmax, int d, double tol) {
    g_sub.clear();
    g_group.clear();
    bool split = false;
    for (const RankCfg& r : ranks) {
        const int on = r.split ? 1 : 0;
        g_sub.push_back({r.threads, r.depth, on, -on});
        g_group.push_back(r.group);
        split = split || r.split == 1;
    }
    const int nr = (int)ranks.size();
    std::vector<std::vector<std::string>> logs(nr);
    if (!split) {
        for (int i = 0; i < nr; ++i) {
            g_rank = i;
            logs[i] = run_rank(ranks[i], kmax, d, tol, i, nr);
        }
    } else {
        // the evaluation split: ranks wait for each other's results, so they run concurrently
        // (each on its own thread with its own stand-in decomposition), through the real mailbox
        char key[64];
        snprintf(key, sizeof key, "xsim_%d_%s", (int)getpid(), name);
        for (char* p = key; *p; ++p)
            if (!isalnum((unsigned char)*p)) *p = '_';
        g_key = key;
        std::vector<std::thread> th;
        for (int i = 0; i < nr; ++i) th.emplace_back([&, i] { logs[i] = run_rank(ranks[i], kmax, d, tol, i, nr); });
        for (auto& t : th) t.join();
    }
    bool same = true;
    for (size_t i = 1; i < logs.size(); ++i) same = same && logs[i] == logs[0];
    std::string first;
    for (const std::string& s : logs[0]) first += s + " ";
    printf("JOB %s ranks=%zu identical=%d calls=%zu first=%s\n", name, ranks.size(), same ? 1 : 0, logs[0].size(),
           first.c_str());
    if (!same)
        for (size_t i = 0; i < logs.size(); ++i) {
            std::string l;
            for (const std::string& s : logs[i]) l += s + " ";
            printf("  rank %zu: %s\n", i, l.c_str());
        }
    return same ? 0 : 1;
}

int main() {
    const char* e = getenv("XSCHED_SIM_LOCAL");
    g_local = e && e[0] == '1';
    int bad = 0;
    const int K = 50, d = 8;
    // the cases of ADVICE r2: an nf = 0 rank beside one-sweep ranks, different thread
    // counts (hence depths) and a different TKHIP_XCH_GROUP on one rank
    bad += run_job("onesweep+empty", {{ONESWEEP, 4, 2, 4}, {EMPTY, 4, 2, 4}}, K, d, 0.0);
    bad += run_job("threads", {{ONESWEEP, 1, 2, 4}, {ONESWEEP, 8, 2, 4}, {CGS2, 3, 5, 4}}, K, d, 0.0);
    bad += run_job("group-env", {{ONESWEEP, 4, 2, 4}, {CGS2, 4, 2, 8}, {EMPTY, 2, 2, 1}}, K, d, 0.0);
    bad += run_job("converged", {{ONESWEEP, 4, 2, 4}, {EMPTY, 8, 3, 4}, {CGS2, 1, 2, 16}}, K, d, 1.0);
    bad += run_job("group1", {{ONESWEEP, 2, 2, 1}, {CGS2, 2, 2, 1}}, 12, 3, 0.0);
    // odd nmax, no convergence: the last one-sweep step leaves its column pending
    bad += run_job("odd-nonconv", {{ONESWEEP, 4, 2, 4}, {ONESWEEP, 2, 3, 4}, {EMPTY, 4, 2, 4}}, 49, d, 0.0);
    bad += run_job("mixed8", {{ONESWEEP, 8, 2, 4}, {ONESWEEP, 8, 2, 4}, {CGS2, 8, 2, 4}, {EMPTY, 8, 2, 4},
                              {ONESWEEP, 1, 9, 4}, {CGS2, 2, 2, 4}, {EMPTY, 5, 2, 2}, {ONESWEEP, 3, 4, 7}},
                   K, d, 0.0);
    // the evaluation split (tk_solver_share): every rank evaluates 1 / nranks of the
    // iterations and reads the others' from the mailbox -- same all-reduces, same outcome
    if (!g_local) {
        bad += run_job("split2", {{ONESWEEP, 4, 2, 4, 1}, {ONESWEEP, 2, 3, 4, 1}}, K, d, 0.0);
        bad += run_job("split-converged", {{ONESWEEP, 4, 2, 4, 1}, {EMPTY, 8, 3, 4, 1}, {CGS2, 1, 2, 16, 1}}, K, d, 1.0);
        bad += run_job("split8", {{ONESWEEP, 8, 2, 4, 1}, {ONESWEEP, 8, 2, 4, 1}, {CGS2, 8, 2, 4, 1}, {EMPTY, 8, 2, 4, 1},
                                  {ONESWEEP, 1, 9, 4, 1}, {CGS2, 2, 2, 4, 1}, {EMPTY, 5, 2, 2, 1}, {ONESWEEP, 3, 4, 7, 1}},
                       K, d, 0.0);
        // one rank with a results source, one without: nobody splits (the agreed flag), the
        // same sequence
        bad += run_job("split-partial", {{ONESWEEP, 4, 2, 4, 0}, {ONESWEEP, 4, 2, 4, 2}}, K, d, 0.0);
    }
    printf("RESULT %s\n", bad ? "MISMATCH" : "OK");
    return bad ? 1 : 0;
}
