// tk_solver.cpp -- the host side of tensorkrylov!'s iteration loop, native
// (src/tensor_krylov_method.jl:63-118; SURVEY.md 8(b) "the C++ host driver", 8(f) rows 1-2).
//
// Per iteration k the reference's host work is: apply the step's results to H_s / b~_s
// (orthonormalize! + update_rhs!), solve the compressed system, evaluate the residual, record
// the orthogonality of V_1, test convergence.  Everything except the record bookkeeping is a
// pure function of (H_s[1:k, 1:k], H_s[k+1, k], b~_s[1:k], the exp-sum table of k): steps
// after k only write H columns >= k, rows >= k and b~ entries >= k.  So the driver
// (tk_solver_run) applies records in order on the calling thread and hands each iteration's
// evaluation to a pool of worker threads: iterations k, k+1, ... are evaluated concurrently
// while the GPU runs further steps ahead, and results are consumed in order -- every
// iterate is bitwise the one a sequential loop computes (the worker count changes only
// throughput).  The spectral bounds and exp-sum ranks/coefficients depend on A and tol
// only; the caller passes them per k (tk_solver_create).
#include <fcntl.h>
#include <math.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <stdio.h>
#include <stdlib.h>

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/tk.h"
#include "tk_host.h"

using namespace tkh;

tk_status tk_fail_internal(int code, const char* msg);   // tk_abi.cpp: tk_last_error()'s store

#define TK_API_BEGIN try {
#define TK_API_END                                                                            \
    }                                                                                         \
    catch (const std::bad_alloc&) { return tk_fail_internal(TK_ERR_ALLOC, "host allocation failed"); } \
    catch (...) { return tk_fail_internal(TK_ERR_INTERNAL, "unknown C++ exception"); }

namespace {

struct IterResult {
    double t0 = -1.0, t1 = -1.0;   // evaluation start / end, steady_clock seconds (TKHIP_SOLVER_TRACE)
    int k = 0;
    int status = TK_OK;           // TK_OK, TK_BREAKDOWN or TK_ERR_STATE (eigen/expm failure)
    double r_comp = 0.0, r_norm = 0.0, rel = 0.0, orth = 0.0;
    Vec lam, Y;                   // lambda (t), Y [d][t][k]
};

// ------------------------------------------------------------------ worker pool
// Idle workers block (the box's CPU share is a cgroup quota: spinning threads would spend
// it); a job is handed over under the worker's mutex, its completion under the pool's.  The
// threads belong to the solver: started ahead of the loop (tk_solver_prepare, the driver's
// setup) or by its first run, kept until tk_solver_destroy.
struct Worker {
    std::mutex mu;
    std::condition_variable cv;
    int job = 0;                  // iteration to evaluate, 0 = idle, -1 = exit
    IterResult res;
    Work ws;
    std::thread th;
};

struct Pool {
    std::mutex mu;
    std::condition_variable cv;
    std::vector<int> done;        // per worker: iteration whose result is ready
};

// Helper threads for the last iterations' evaluations (tkh::ParFor): persistent, so a split
// costs a wake-up, not a thread start (a std::thread per split cost more than it saved:
// C4 tail 476 vs 227 us, profiles/r04/e2e_traces_tail_threads_ab.txt).  Idle helpers block;
// while `hot` (set by the loop when the tail iterations are dispatched) they spin instead,
// so the split finds them running.  One split at a time: a second caller (two workers in
// the tail together) runs its tasks itself.
class Helpers : public ParFor {
  public:
    explicit Helpers(int nh) {
        for (int i = 0; i < nh; ++i) th_.emplace_back([this] { loop(); });
    }
    ~Helpers() override {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_.store(true);
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return (int)th_.size(); }
    void set_hot(bool h) {
        if (hot_.exchange(h) == h || !h) return;
        {
            std::lock_guard<std::mutex> lk(mu_);
            ++wake_;
        }
        cv_.notify_all();
    }
    void run(int n, void (*fn)(void*, int), void* ctx) override {
        std::unique_lock<std::mutex> own(call_mu_, std::try_to_lock);
        if (!own.owns_lock() || th_.empty()) {
            for (int i = 0; i < n; ++i) fn(ctx, i);
            return;
        }
        Job j;
        j.fn = fn;
        j.ctx = ctx;
        j.n = n;
        j.left.store(n, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> lk(mu_);
            cur_ = &j;
            posted_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        take(j);
        while (j.left.load(std::memory_order_acquire) > 0) _mm_pause();
        {
            std::lock_guard<std::mutex> lk(mu_);
            cur_ = nullptr;
        }
        // (a helper that picked the job up may still be between its last task and leaving)
        while (j.refs.load(std::memory_order_acquire) > 0) _mm_pause();
    }

  private:
    struct Job {
        void (*fn)(void*, int) = nullptr;
        void* ctx = nullptr;
        int n = 0;
        std::atomic<int> next{0}, left{0}, refs{0};
    };
    static void take(Job& j) {
        for (int i; (i = j.next.fetch_add(1, std::memory_order_relaxed)) < j.n;) {
            j.fn(j.ctx, i);
            j.left.fetch_sub(1, std::memory_order_release);
        }
    }
    void loop() {
        unsigned seen = 0, wseen = 0;
        for (;;) {
            for (int spin = 0;;) {
                if (quit_.load(std::memory_order_acquire)) return;
                if (posted_.load(std::memory_order_acquire) != seen) break;
                if (hot_.load(std::memory_order_relaxed) || ++spin < 4096) {
                    _mm_pause();
                    continue;
                }
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return quit_.load() || posted_.load() != seen || wake_ != wseen; });
                wseen = wake_;
                spin = 0;
            }
            Job* j;
            {
                std::lock_guard<std::mutex> lk(mu_);
                seen = posted_.load(std::memory_order_relaxed);
                j = cur_;
                if (j) j->refs.fetch_add(1, std::memory_order_relaxed);
            }
            if (!j) continue;
            take(*j);
            j->refs.fetch_sub(1, std::memory_order_release);
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_, call_mu_;
    std::condition_variable cv_;
    Job* cur_ = nullptr;
    std::atomic<unsigned> posted_{0};
    std::atomic<bool> hot_{false}, quit_{false};
    unsigned wake_ = 0;
};

// TKHIP_SOLVER_TAIL_THREADS: tasks (1..4) the last two iterations' evaluations split into.
// Default 3 (2 helpers): C4's tail 240-316 -> 115-138 us, end-to-end 0.94 -> 0.96 of the
// device rate; no change where the host is throughput-bound (C4 emulated N = 8)
// (profiles/r04/e2e/native_orth_tail_ab.txt, tail_helpers_ab_traced.txt)
static int tail_threads() {
    static const int v = [] {
        const char* e = getenv("TKHIP_SOLVER_TAIL_THREADS");
        return e ? std::max(1, std::min(4, atoi(e))) : 3;
    }();
    return v;
}

// TKHIP_SOLVER_TAIL_ITERS: how many of the last iterations may split over the helpers.  2; 8
// (with the helpers spinning for all 8) lets the evaluations that pile up behind a short sweep
// use them too (C4 emulated N = 8: 0.79-0.84 -> 0.84-0.89 of the device rate) but cost the
// N = 1 lines 1-2 % (C4 0.960 -> 0.948; profiles/r04/e2e/host_avx512_tail_iters_ab.txt)
static int tail_iters() {
    static const int v = [] {
        const char* e = getenv("TKHIP_SOLVER_TAIL_ITERS");
        return e ? std::max(1, std::min(64, atoi(e))) : 2;
    }();
    return v;
}

// TKHIP_SOLVER_HOT_ITERS: from the dispatch of iteration klast - this on, the helpers spin
// instead of blocking (earlier splits wake them through their condition variable)
static int hot_iters() {
    static const int v = [] {
        const char* e = getenv("TKHIP_SOLVER_HOT_ITERS");
        return e ? std::max(1, std::min(64, atoi(e))) : 2;
    }();
    return v;
}

// ------------------------------------------------------------------ evaluation split
// With several ranks every rank holds the same host mirror (the records all-reduce gives each
// every factor's record), so iteration k's evaluation is the same pure function on every
// rank: rank (k mod nranks) evaluates it and the others read its result.  The
// results travel through a node-local mailbox -- one POSIX shared-memory file per job, one
// 64-byte entry per iteration, a generation word written last -- not through the records
// all-reduce: a result posted in a later step's slot would reach the other ranks only with
// that step's records, i.e. every convergence / breakdown decision L steps late, and the last
// L iterations would need an extra collective.  The mailbox costs a cache line per iteration.
struct MailHeader {
    uint64_t magic, nranks, kmax, attached;
    uint64_t pad[4];
};
struct MailEntry {                 // one per iteration k (index k)
    uint64_t gen;                  // written last (release): the run this entry belongs to
    double rc, rn, rel, orth;
    int64_t status;
    uint64_t pad[2];
};
static_assert(sizeof(MailHeader) == 64 && sizeof(MailEntry) == 64, "one cache line each");
static const uint64_t MAIL_MAGIC = 0x746b6869705f6576ull;   // "tkhip_ev"

struct Share {
    int nranks = 1, rank = 0;
    MailHeader* hdr = nullptr;     // mailbox (real ranks)
    MailEntry* ent = nullptr;
    size_t bytes = 0;
    std::vector<double> table;     // emulation: a full run's results [k-1][6] (tk_solver_results)
    uint64_t gen = 0;              // this run's generation (every rank counts runs alike)
    int last_k = 1 << 30;          // (tk_solver_evaluate_shared: a new generation when k restarts)
    bool on() const { return nranks > 1; }
    bool owner(int k) const { return nranks <= 1 || k % nranks == rank; }
};

// per-iteration results of the last run, [k-1][6] = r_comp, r_norm, rel, orth, status, eval us
enum { RES_RC, RES_RN, RES_REL, RES_ORTH, RES_ST, RES_US, RES_N };

}  // namespace

struct tk_solver {
    int method, d, kmax, KP, KC, m, symmetric;
    double bnorm;
    std::vector<double> lmin;
    std::vector<int> rank, roff;
    std::vector<double> alpha, omega;
    std::vector<double> H;        // [s][c * KP + r]  (H_s, (kmax+2) x (kmax+1), column-major)
    std::vector<double> bt;       // [s][c]
    std::vector<double> gram0;    // factor 0's Gram rows: [c * KC + i], i <= c
    bool gram_tracked = false;    // factor 0's records carry Gram rows (else: a deferred Gram,
                                  // tk_decomp_gram; orthogonality_data is filled by the caller)
    std::vector<double> loss;     // [s][j] LanczosReorth loss of step j
    std::vector<unsigned char> reorth;
    IterResult last;
    Work ws;
    // emulation overlay (bench --emulate-ranks): rows of factors outside [ov_first,
    // ov_first + ov_nf) are taken from records recorded by a full run, [slot][d][m]
    std::vector<double> overlay;
    int ov_first = 0, ov_nf = 0;
    Pool pool;
    std::vector<std::unique_ptr<Worker>> workers;
    std::unique_ptr<Helpers> helpers;   // (tail_threads() > 1)
    Share share;
    std::vector<double> results;        // [kmax][RES_N] of the last run (NaN: not consumed)
};

static void mail_post(tk_solver* sv, const IterResult& r) {
    MailEntry* e = sv->share.ent;
    if (!e || r.k < 0 || r.k > sv->kmax) return;
    e += r.k;
    e->rc = r.r_comp;
    e->rn = r.r_norm;
    e->rel = r.rel;
    e->orth = r.orth;
    e->status = r.status;
    __atomic_store_n(&e->gen, sv->share.gen, __ATOMIC_RELEASE);
}

static double wait_limit_solver_s() {
    const char* e = getenv("TKHIP_WAIT_S");
    const double v = e ? atof(e) : 120.0;
    return v > 0 ? v : 120.0;
}

// iteration k's result from its owner: the mailbox (bounded by TKHIP_WAIT_S), or in
// emulation the full run's table, released no earlier than the owner would have had it (the
// record's arrival here + the owner's evaluation time in that run)
static tk_status mail_take(tk_solver* sv, int k, IterResult& out, std::chrono::steady_clock::time_point t_rec) {
    Share& sh = sv->share;
    out.k = k;
    out.lam.clear();
    out.Y.clear();
    if (sh.ent) {
        const MailEntry* e = sh.ent + k;
        const auto t0 = std::chrono::steady_clock::now();
        const double lim = wait_limit_solver_s();
        for (long spins = 0; __atomic_load_n(&e->gen, __ATOMIC_ACQUIRE) != sh.gen; ++spins) {
            _mm_pause();
            if ((spins & 1023) == 1023) {
                if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim) {
                    char b[160];
                    snprintf(b, sizeof b, "evaluation split: rank %d never published iteration %d (%.0f s, TKHIP_WAIT_S)",
                             k % sh.nranks, k, lim);
                    return tk_fail_internal(TK_ERR_RCCL, b);
                }
                std::this_thread::yield();
            }
        }
        out.r_comp = e->rc;
        out.r_norm = e->rn;
        out.rel = e->rel;
        out.orth = e->orth;
        out.status = (int)e->status;
        return TK_OK;
    }
    const double* r = &sh.table[(size_t)(k - 1) * RES_N];
    const auto ready = t_rec + std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                                   std::chrono::duration<double, std::micro>(std::max(0.0, r[RES_US])));
    while (std::chrono::steady_clock::now() < ready) _mm_pause();
    out.r_comp = r[RES_RC];
    out.r_norm = r[RES_RN];
    out.rel = r[RES_REL];
    out.orth = r[RES_ORTH];
    out.status = (int)r[RES_ST];
    return TK_OK;
}

static void share_close(Share& sh) {
    if (sh.hdr) munmap(sh.hdr, sh.bytes);
    sh.hdr = nullptr;
    sh.ent = nullptr;
    sh.table.clear();
    sh.nranks = 1;
    sh.rank = 0;
}

static void apply_record(tk_solver* sv, int j, const double* rec) {
    const int kmax = sv->kmax, m = sv->m, KP = sv->KP, KC = sv->KC;
    std::vector<double> merged;
    if (!sv->overlay.empty()) {
        merged.assign(rec, rec + (size_t)sv->d * m);
        const double* ov = &sv->overlay[(size_t)(j + 1) * sv->d * m];
        for (int s = 0; s < sv->d; ++s)
            if (s < sv->ov_first || s >= sv->ov_first + sv->ov_nf)
                memcpy(&merged[(size_t)s * m], ov + (size_t)s * m, m * sizeof(double));
        rec = merged.data();
    }
    const int o_gram = kmax + 2, o_bt = 2 * kmax + 4, o_col = 2 * kmax + 5, o_loss = 2 * kmax + 7,
              o_flag = 2 * kmax + 8, o_tracked = 2 * kmax + 9;
    for (int s = 0; s < sv->d; ++s) {
        const double* r = rec + (size_t)s * m;
        double* H = &sv->H[(size_t)s * KP * KC];
        auto h = [&](int row, int col) -> double& { return H[(size_t)col * KP + row]; };
        if (j >= 0) {
            if (sv->method == TK_ARNOLDI) {                       // H[:, j] (src/orthogonal_bases.jl:22-36)
                for (int i = 0; i <= j + 1; ++i) h(i, j) = r[i];
            } else {
                double beta;
                if (sv->method == TK_LANCZOS_REORTH) sv->loss[(size_t)s * KC + j] = r[o_loss];
                if (sv->method == TK_LANCZOS_REORTH && r[o_flag] > 0) {   // :123-131
                    sv->reorth[(size_t)s * KC + j] = 1;
                    for (int i = 0; i <= j + 1; ++i) h(i, j) = r[i];
                    beta = h(j + 1, j);
                    for (int i = 0; i < std::max(j - 1, 0); ++i) h(i, j) = 0.0;
                } else {                                          // TTR :50
                    h(j, j) = r[j];
                    beta = r[j + 1];
                }
                h(j + 1, j) = beta;                               // update_subdiagonals!
                if (j + 1 < KC) h(j, j + 1) = beta;
            }
        }
        const int c = (int)lround(r[o_col]);
        if (c >= 0 && c < KC) {
            sv->bt[(size_t)s * KC + c] = r[o_bt];                 // update_rhs! (src/utils.jl:466-476)
            if (s == 0 && r[o_tracked] > 0) {
                sv->gram_tracked = true;
                for (int i = 0; i <= c; ++i) sv->gram0[(size_t)c * KC + i] = r[o_gram + i];
            }
        }
    }
}

// iteration k (2 <= k <= kmax): compressed solve, residual, orthogonality of V_1
static void evaluate(const tk_solver* sv, int k, IterResult& out, Work& ws) {
    const int d = sv->d, KP = sv->KP, KC = sv->KC;
    const int t = sv->rank[k - 1];
    const double* al = &sv->alpha[sv->roff[k - 1]];
    const double* om = &sv->omega[sv->roff[k - 1]];
    out.k = k;
    out.status = TK_OK;
    out.lam.resize(t);
    out.Y.resize((size_t)d * t * k);
    if (!compressed_solve(d, k, sv->H.data(), KP, sv->symmetric, sv->bt.data(), KC, t, al, om, sv->lmin[k - 1],
                          out.lam.data(), out.Y.data(), ws)) {
        out.status = TK_ERR_STATE;
        return;
    }
    double sub[64];
    std::vector<double> subv;
    double* sp = sub;
    if (d > 64) {
        subv.resize(d);
        sp = subv.data();
    }
    for (int s = 0; s < d; ++s) sp[s] = sv->H[(size_t)s * KP * KC + (size_t)(k - 1) * KP + k];   // H_s[k+1, k]
    if (residual(d, k, t, sv->H.data(), KP, (size_t)KP * KC, out.lam.data(), out.Y.data(), sp, sv->bt.data(), KC,
                 sv->bnorm, &out.r_comp, &out.r_norm, ws)) {
        out.status = TK_BREAKDOWN;
        return;
    }
    out.rel = out.r_norm / sv->bnorm;                              // :99
    // orthogonality_loss(V_1, k) = norm(V'V - I) from the lower Gram rows (:103); NaN when
    // factor 0's Gram is deferred (the caller fills orthogonality_data from tk_decomp_gram)
    if (!sv->gram_tracked) {
        out.orth = NAN;
        return;
    }
    double acc = 0.0;
    for (int c = 0; c < k; ++c) {
        const double* g = &sv->gram0[(size_t)c * KC];
        const double dd = g[c] - 1.0;
        double off = 0.0;
        for (int i = 0; i < c; ++i) off += g[i] * g[i];
        acc += dd * dd + 2.0 * off;
    }
    out.orth = sqrt(acc);
}

static void worker_loop(tk_solver* sv, int w, Worker* wkp) {
    Worker& wk = *wkp;
    for (;;) {
        int k;
        {
            std::unique_lock<std::mutex> lk(wk.mu);
            wk.cv.wait(lk, [&] { return wk.job != 0; });
            k = wk.job;
        }
        if (k < 0) return;
        const double tb = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        evaluate(sv, k, wk.res, wk.ws);
        wk.res.t0 = tb;
        wk.res.t1 = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
        if (sv->share.ent) mail_post(sv, wk.res);   // (split: the other ranks read it at once)
        {
            std::lock_guard<std::mutex> lk(wk.mu);
            wk.job = 0;
        }
        {
            std::lock_guard<std::mutex> lk(sv->pool.mu);
            sv->pool.done[w] = k;
        }
        sv->pool.cv.notify_all();
    }
}

// at least P worker threads (only between runs: no job is in flight)
static void start_workers(tk_solver* sv, int P) {
    {
        std::lock_guard<std::mutex> lk(sv->pool.mu);
        if ((int)sv->pool.done.size() < P) sv->pool.done.resize(P, 0);
    }
    while ((int)sv->workers.size() < P) {
        Worker* wk = new Worker();
        sv->workers.emplace_back(wk);
        wk->th = std::thread(worker_loop, sv, (int)sv->workers.size() - 1, wk);
    }
    if (tail_threads() > 1 && !sv->helpers) sv->helpers.reset(new Helpers(tail_threads() - 1));
}

static void stop_workers(tk_solver* sv) {
    for (auto& wk : sv->workers) {
        {
            std::lock_guard<std::mutex> lk(wk->mu);
            wk->job = -1;
        }
        wk->cv.notify_one();
    }
    for (auto& wk : sv->workers) wk->th.join();
    sv->workers.clear();
    sv->helpers.reset();
}

// norm(G[:k, :k] - I), k = 1..K (G column-major, lower triangle): tk_solver_evaluate's sum
static void orth_losses(int K, const double* G, int ld, double* out) {
    double acc = 0.0;
    for (int c = 0; c < K; ++c) {
        const double dd = G[(size_t)c * ld + c] - 1.0;
        double off = 0.0;
        for (int i = 0; i < c; ++i) off += G[(size_t)i * ld + c] * G[(size_t)i * ld + c];
        acc += dd * dd + 2.0 * off;
        out[c] = sqrt(acc);
    }
}

extern "C" {

tk_status tk_orthogonality_losses(int K, const double* G, double* out) { TK_API_BEGIN
    if (K < 0 || (K > 0 && (!G || !out))) return tk_fail_internal(TK_ERR_ARG, "tk_orthogonality_losses: bad argument");
    orth_losses(K, G, K, out);
    return TK_OK;
    TK_API_END
}

tk_status tk_solver_prepare(tk_solver* sv, int nthreads) { TK_API_BEGIN
    if (!sv || nthreads < 1) return tk_fail_internal(TK_ERR_ARG, "tk_solver_prepare: bad argument");
    start_workers(sv, std::min(nthreads, 64));
    return TK_OK;
    TK_API_END
}

tk_status tk_solver_create(int method, int d, int kmax, int symmetric, double b_norm, const double* lmin,
                           const int* rank, const double* alpha, const double* omega, tk_solver** out) { TK_API_BEGIN
    if (!out || d < 1 || kmax < 1 || !lmin || !rank || !alpha || !omega || method < 0 || method > 2)
        return tk_fail_internal(TK_ERR_ARG, "tk_solver_create: bad argument");
    tk_solver* sv = new tk_solver();
    sv->method = method;
    sv->d = d;
    sv->kmax = kmax;
    sv->KP = kmax + 2;
    sv->KC = kmax + 1;
    sv->m = tk_record_len(kmax);
    sv->symmetric = symmetric;
    sv->bnorm = b_norm;
    sv->lmin.assign(lmin, lmin + kmax);
    sv->rank.assign(rank, rank + kmax);
    sv->roff.assign(kmax, 0);
    int tot = 0;
    for (int k = 0; k < kmax; ++k) {
        if (rank[k] < 0) {
            delete sv;
            return tk_fail_internal(TK_ERR_ARG, "tk_solver_create: negative rank");
        }
        sv->roff[k] = tot;
        tot += rank[k];
    }
    sv->alpha.assign(alpha, alpha + tot);
    sv->omega.assign(omega, omega + tot);
    sv->H.assign((size_t)d * sv->KP * sv->KC, 0.0);
    sv->bt.assign((size_t)d * sv->KC, 0.0);
    sv->gram0.assign((size_t)sv->KC * sv->KC, 0.0);
    sv->loss.assign((size_t)d * sv->KC, 0.0);
    sv->reorth.assign((size_t)d * sv->KC, 0);
    sv->results.assign((size_t)kmax * RES_N, NAN);
    *out = sv;
    return TK_OK;
    TK_API_END
}

tk_status tk_solver_overlay(tk_solver* sv, int first, int nf, const double* records) { TK_API_BEGIN
    if (!sv || first < 0 || nf < 0 || first + nf > sv->d) return tk_fail_internal(TK_ERR_ARG, "tk_solver_overlay: bad argument");
    if (!records) {
        sv->overlay.clear();
        return TK_OK;
    }
    sv->overlay.assign(records, records + (size_t)(sv->kmax + 2) * sv->d * sv->m);
    sv->ov_first = first;
    sv->ov_nf = nf;
    return TK_OK;
    TK_API_END
}

tk_status tk_solver_destroy(tk_solver* sv) {
    if (!sv) return TK_OK;
    stop_workers(sv);
    share_close(sv->share);
    delete sv;
    return TK_OK;
}

tk_status tk_solver_apply(tk_solver* sv, int j, const double* rec) { TK_API_BEGIN
    if (!sv || !rec || j < -1 || j >= sv->kmax) return tk_fail_internal(TK_ERR_ARG, "tk_solver_apply: bad argument");
    apply_record(sv, j, rec);
    return TK_OK;
    TK_API_END
}

tk_status tk_solver_evaluate(tk_solver* sv, int k, double* out4) { TK_API_BEGIN
    if (!sv || !out4 || k < 2 || k > sv->kmax || sv->rank[k - 1] < 1)
        return tk_fail_internal(TK_ERR_ARG, "tk_solver_evaluate: bad argument");
    // (TKHIP_EVAL_THREADS: tasks of this single evaluation, on helper threads -- timing tools)
    if (const char* e = getenv("TKHIP_EVAL_THREADS")) {
        sv->ws.nthreads = std::max(1, std::min(4, atoi(e)));
        if (sv->ws.nthreads > 1 && !sv->helpers) sv->helpers.reset(new Helpers(sv->ws.nthreads - 1));
        sv->ws.par = sv->helpers.get();
    }
    evaluate(sv, k, sv->last, sv->ws);
    out4[0] = sv->last.r_comp;
    out4[1] = sv->last.r_norm;
    out4[2] = sv->last.rel;
    out4[3] = sv->last.orth;
    if (sv->last.status == TK_ERR_STATE) return tk_fail_internal(TK_ERR_STATE, "compressed solve failed (eigen / expm)");
    return sv->last.status;
    TK_API_END
}

int tk_solver_rank(tk_solver* sv, int k) { return (sv && k >= 1 && k <= sv->kmax) ? sv->rank[k - 1] : -1; }

tk_status tk_solver_solution(tk_solver* sv, int k, double* lambda_out, double* Y_out) { TK_API_BEGIN
    if (!sv || sv->last.k != k || !lambda_out || !Y_out)
        return tk_fail_internal(TK_ERR_STATE, "tk_solver_solution: iteration k was not the last evaluated");
    memcpy(lambda_out, sv->last.lam.data(), sv->last.lam.size() * sizeof(double));
    memcpy(Y_out, sv->last.Y.data(), sv->last.Y.size() * sizeof(double));
    return TK_OK;
    TK_API_END
}

tk_status tk_solver_state(tk_solver* sv, double* H_out, double* bt_out, double* gram0_out) { TK_API_BEGIN
    if (!sv) return tk_fail_internal(TK_ERR_ARG, "NULL solver");
    const int KP = sv->KP, KC = sv->KC;
    if (H_out)   // [s][r][c] row-major (the host mirror's layout)
        for (int s = 0; s < sv->d; ++s)
            for (int r = 0; r < KP; ++r)
                for (int c = 0; c < KC; ++c)
                    H_out[((size_t)s * KP + r) * KC + c] = sv->H[(size_t)s * KP * KC + (size_t)c * KP + r];
    if (bt_out) memcpy(bt_out, sv->bt.data(), sv->bt.size() * sizeof(double));
    if (gram0_out) memcpy(gram0_out, sv->gram0.data(), sv->gram0.size() * sizeof(double));
    return TK_OK;
    TK_API_END
}

tk_status tk_solver_share(tk_solver* sv, const char* key, int nranks, int rank) { TK_API_BEGIN
    if (!sv || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !key))
        return tk_fail_internal(TK_ERR_ARG, "tk_solver_share: bad argument");
    share_close(sv->share);
    if (nranks == 1) return TK_OK;
    for (const char* p = key; *p; ++p)
        if (!((*p >= '0' && *p <= '9') || (*p >= 'a' && *p <= 'z') || (*p >= 'A' && *p <= 'Z') || *p == '_') ||
            p - key > 96)
            return tk_fail_internal(TK_ERR_ARG, "tk_solver_share: key must be [0-9A-Za-z_]{1,96}");
    char name[160];
    snprintf(name, sizeof name, "/dev/shm/tkhip_ev_%s", key);
    const size_t bytes = sizeof(MailHeader) + (size_t)(sv->kmax + 2) * sizeof(MailEntry);
    const double lim = wait_limit_solver_s();
    const auto t0 = std::chrono::steady_clock::now();
    auto expired = [&] { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim; };
    char msg[256];
    int fd = -1;
    if (rank == 0) {
        // create under a temporary name, initialise, then publish by rename (no rank maps a
        // half-built file); unlinked once every rank has attached
        char tmp[192];
        snprintf(tmp, sizeof tmp, "%s.%d.tmp", name, (int)getpid());
        fd = open(tmp, O_RDWR | O_CREAT | O_EXCL, 0600);
        if (fd < 0 || ftruncate(fd, (off_t)bytes) != 0) {
            if (fd >= 0) close(fd), unlink(tmp);
            snprintf(msg, sizeof msg, "tk_solver_share: cannot create %s", tmp);
            return tk_fail_internal(TK_ERR_STATE, msg);
        }
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (m == MAP_FAILED) {
            unlink(tmp);
            return tk_fail_internal(TK_ERR_STATE, "tk_solver_share: mmap failed");
        }
        memset(m, 0, bytes);
        MailHeader* h = (MailHeader*)m;
        h->magic = MAIL_MAGIC;
        h->nranks = (uint64_t)nranks;
        h->kmax = (uint64_t)sv->kmax;
        __atomic_store_n(&h->attached, 1, __ATOMIC_RELEASE);
        if (rename(tmp, name) != 0) {
            munmap(m, bytes);
            unlink(tmp);
            snprintf(msg, sizeof msg, "tk_solver_share: cannot publish %s", name);
            return tk_fail_internal(TK_ERR_STATE, msg);
        }
        while (__atomic_load_n(&h->attached, __ATOMIC_ACQUIRE) < (uint64_t)nranks) {
            if (expired()) {
                unlink(name);
                munmap(m, bytes);
                snprintf(msg, sizeof msg, "tk_solver_share: %d of %d ranks attached to %s within %.0f s (TKHIP_WAIT_S)",
                         (int)__atomic_load_n(&h->attached, __ATOMIC_ACQUIRE), nranks, name, lim);
                return tk_fail_internal(TK_ERR_RCCL, msg);
            }
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        unlink(name);   // every rank holds its mapping: nothing is left in /dev/shm
        sv->share.hdr = h;
    } else {
        while ((fd = open(name, O_RDWR)) < 0) {
            if (expired()) {
                snprintf(msg, sizeof msg, "tk_solver_share: rank 0 never published %s within %.0f s (TKHIP_WAIT_S)", name, lim);
                return tk_fail_internal(TK_ERR_RCCL, msg);
            }
            std::this_thread::sleep_for(std::chrono::microseconds(100));
        }
        struct stat st;
        void* m = (fstat(fd, &st) == 0 && (size_t)st.st_size == bytes)
                      ? mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0) : MAP_FAILED;
        close(fd);
        MailHeader* h = (MailHeader*)m;
        if (m == MAP_FAILED || h->magic != MAIL_MAGIC || h->nranks != (uint64_t)nranks || h->kmax != (uint64_t)sv->kmax) {
            if (m != MAP_FAILED) munmap(m, bytes);
            snprintf(msg, sizeof msg, "tk_solver_share: %s does not describe this job (%d ranks, kmax %d)", name, nranks,
                     sv->kmax);
            return tk_fail_internal(TK_ERR_STATE, msg);
        }
        __atomic_fetch_add(&h->attached, 1, __ATOMIC_ACQ_REL);
        sv->share.hdr = h;
    }
    sv->share.bytes = bytes;
    sv->share.ent = (MailEntry*)(sv->share.hdr + 1);
    sv->share.nranks = nranks;
    sv->share.rank = rank;
    return TK_OK;
    TK_API_END
}

tk_status tk_solver_share_emulated(tk_solver* sv, int nranks, int rank, const double* results) { TK_API_BEGIN
    if (!sv || nranks < 1 || rank < 0 || rank >= nranks || (nranks > 1 && !results))
        return tk_fail_internal(TK_ERR_ARG, "tk_solver_share_emulated: bad argument");
    share_close(sv->share);
    if (nranks == 1) return TK_OK;
    sv->share.table.assign(results, results + (size_t)sv->kmax * RES_N);
    sv->share.nranks = nranks;
    sv->share.rank = rank;
    return TK_OK;
    TK_API_END
}

tk_status tk_solver_results(tk_solver* sv, double* out) { TK_API_BEGIN
    if (!sv || !out) return tk_fail_internal(TK_ERR_ARG, "tk_solver_results: bad argument");
    memcpy(out, sv->results.data(), sv->results.size() * sizeof(double));
    return TK_OK;
    TK_API_END
}

tk_status tk_solver_evaluate_shared(tk_solver* sv, int k, double* out4) { TK_API_BEGIN
    if (!sv || !out4 || k < 2 || k > sv->kmax || sv->rank[k - 1] < 1)
        return tk_fail_internal(TK_ERR_ARG, "tk_solver_evaluate_shared: bad argument");
    Share& sh = sv->share;
    if (!sh.on()) return tk_solver_evaluate(sv, k, out4);
    if (k <= sh.last_k) ++sh.gen;   // a new loop (every rank restarts at the same k)
    sh.last_k = k;
    IterResult r;
    if (sh.owner(k)) {
        evaluate(sv, k, sv->last, sv->ws);
        mail_post(sv, sv->last);
        r = sv->last;
    } else {
        tk_status st = mail_take(sv, k, r, std::chrono::steady_clock::now());
        if (st) return st;
    }
    out4[0] = r.r_comp;
    out4[1] = r.r_norm;
    out4[2] = r.rel;
    out4[3] = r.orth;
    if (r.status == TK_ERR_STATE) return tk_fail_internal(TK_ERR_STATE, "compressed solve failed (eigen / expm)");
    return r.status;
    TK_API_END
}

tk_status tk_solver_run(tk_solver* sv, tk_decomp* dc, double tol, int kfirst, int depth, int nthreads,
                        double* relres, double* projres, double* orth, int* k_end, int* outcome) { TK_API_BEGIN
    if (!sv || !dc || !relres || !projres || !orth || !k_end || !outcome || kfirst < 2)
        return tk_fail_internal(TK_ERR_ARG, "tk_solver_run: bad argument");
    const auto t_entry = std::chrono::steady_clock::now();
    const int kmax = sv->kmax;
    int klast = kmax;   // iterations with a tabulated exp-sum rank
    for (int k = kfirst; k <= kmax; ++k)
        if (sv->rank[k - 1] < 1) {
            klast = k - 1;
            break;
        }
    // every rank must issue the same sequence of steps and record reads (the records
    // all-reduces follow it, tk_xsched.h): agree the worker count and depth (max over ranks)
    // ... and whether the evaluations are split over the ranks: on only if EVERY rank has the
    // mailbox (max of the flag = 1 and max of its negation = 0), so no rank waits for results
    // a rank without one would never post
    Share& sh = sv->share;
    const int son = sh.on() ? 1 : 0;
    int agreed[4] = {std::max(1, std::min(nthreads, 64)), depth, son, -son};
    {
        tk_status st0 = tk_decomp_agree(dc, agreed, 4);
        if (st0) return st0;
    }
    const int P = agreed[0];
    depth = std::max(agreed[1], P + 1);
    const bool split = agreed[2] == 1 && agreed[3] == -1;
    ++sh.gen;                        // (every rank counts its runs alike)
    sh.last_k = 1 << 30;
    // dispatch window: P evaluations in flight per rank; split, each rank owns 1 of NR
    const int NR = split ? sh.nranks : 1;
    const int W = P * NR;
    std::fill(sv->results.begin(), sv->results.end(), NAN);
    *outcome = 0;
    *k_end = klast;
    std::vector<double> rec((size_t)sv->d * sv->m);
    // steps kfirst .. kfirst+depth-1 ahead of the first evaluation (step k is ABI step k-1)
    int next_issue = kfirst;
    auto issue_upto = [&](int kk) -> tk_status {
        for (; next_issue <= std::min(kk, kmax); ++next_issue) {
            tk_status st = tk_decomp_step(dc, next_issue - 1, nullptr);
            if (st) return st;
        }
        return TK_OK;
    };
    // the deferred orthogonality Gram of factor 1 goes to the device right behind the last
    // step (tk_decomp_gram_ahead: no-op on ranks without it), overlapping the host's evaluation
    // of the last iterations; the caller's tk_decomp_gram then only reads it
    bool gram_ahead = false;
    int gram_k = 0;   // columns of the Gram launched ahead (0: none on this rank)
    auto ahead = [&]() -> tk_status {
        if (gram_ahead || next_issue <= kmax) return TK_OK;
        gram_ahead = true;
        return tk_decomp_gram_ahead(dc, &gram_k);
    };
    // ... and once every iteration is dispatched the calling thread reads it (while the
    // workers evaluate the last iterations) and derives orthogonality_data from it
    std::vector<double> gram_loss;
    auto read_gram = [&]() -> tk_status {
        if (gram_k < 1 || sv->gram_tracked || !gram_loss.empty()) return TK_OK;
        std::vector<double> G((size_t)gram_k * gram_k);
        tk_status s2 = tk_decomp_gram(dc, 0, gram_k, G.data());
        if (s2) return s2;
        gram_loss.resize(gram_k);
        orth_losses(gram_k, G.data(), gram_k, gram_loss.data());
        return TK_OK;
    };
    tk_status st = issue_upto(kfirst + depth - 1);
    if (!st) st = ahead();
    if (st) return st;

    start_workers(sv, P);
    auto& workers = sv->workers;
    Pool& pool = sv->pool;
    {
        std::lock_guard<std::mutex> lk(pool.mu);
        for (auto& x : pool.done) x = 0;
    }
    typedef std::chrono::steady_clock clk_t;
    // the last two iterations run when every other evaluation is done or nearly so: their
    // data-parallel parts may be split over the helper threads (Work::nthreads, Work::par;
    // bitwise the same), which spin from the dispatch of iteration klast-2 on
    Helpers* hp = sv->helpers.get();
    const int tail = hp ? tail_threads() : 1;
    struct HotOff {   // (the helpers stop spinning on every way out of the loop, exceptions too)
        Helpers* h;
        ~HotOff() {
            if (h) h->set_hot(false);
        }
    } hot_off{hp};
    // per worker: the iteration submitted and not yet consumed (quiesce waits for its result)
    std::vector<int> inflight(workers.size(), 0);
    // per iteration: the worker evaluating it here (-1: another rank's, read from the mailbox),
    // and when its record was applied here (emulation releases the owner's result from then)
    std::vector<int> wmap(kmax + 2, -1);
    std::vector<clk_t::time_point> t_disp(kmax + 2);
    int nsub = 0;
    auto submit = [&](int w, int k) {
        {
            std::lock_guard<std::mutex> lk(pool.mu);
            pool.done[w] = 0;
        }
        inflight[w] = k;
        // (split: the tail is this rank's last owned iterations, one in NR of the last ones --
        // e.g. C4 at N = 8, rank 7's k = 47 took 127 us on one thread, the loop's end waiting
        // for it; profiles/r05/e2e_trace_split_tail.txt)
        if (hp && k >= klast - hot_iters() * NR) hp->set_hot(true);
        {
            std::lock_guard<std::mutex> lk(workers[w]->mu);
            workers[w]->ws.nthreads = k > klast - tail_iters() * NR ? tail : 1;
            workers[w]->ws.par = hp;
            workers[w]->job = k;
        }
        workers[w]->cv.notify_one();
    };
    auto wait_done = [&](int w, int k) {
        std::unique_lock<std::mutex> lk(pool.mu);
        pool.cv.wait(lk, [&] { return pool.done[w] == k; });
        inflight[w] = 0;
    };
    // the end of a run: jobs still in flight finish (their results are discarded); the
    // threads stay for the next run or tk_solver_destroy.  A worker clears its job before it
    // publishes pool.done (the other order could erase a job submitted in between), so the
    // wait is for the published result itself: a late pool.done write of this run's last
    // iterations must not land after the next run has reset pool.done
    auto quiesce = [&] {
        std::unique_lock<std::mutex> lk(pool.mu);
        for (size_t w = 0; w < inflight.size(); ++w) {
            if (!inflight[w]) continue;
            pool.cv.wait(lk, [&] { return pool.done[w] == inflight[w]; });
            inflight[w] = 0;
        }
    };
    int k_dispatch = kfirst;
    tk_status err = TK_OK;
    // TKHIP_SOLVER_STATS=1: where the calling thread's time goes (stderr)
    const char* est = getenv("TKHIP_SOLVER_STATS");
    const bool stats = est && est[0] == '1';
    typedef std::chrono::steady_clock clk;
    double t_rec = 0, t_issue = 0, t_apply = 0, t_wait = 0;
    auto tp = clk::now();
    auto lap = [&](double& acc) {
        if (!stats) return;
        const auto now = clk::now();
        acc += std::chrono::duration<double, std::micro>(now - tp).count();
        tp = now;
    };
    const auto t_begin = clk::now();
    // TKHIP_SOLVER_TRACE=path: per iteration, microseconds from the loop start at which its
    // record was in hand, its evaluation started and ended (worker clock), and it was consumed
    const char* etr = getenv("TKHIP_SOLVER_TRACE");
    std::vector<double> tr_rec(kmax + 2, -1.0), tr_cons(kmax + 2, -1.0);
    auto since = [&](clk::time_point p) { return std::chrono::duration<double, std::micro>(p - t_begin).count(); };
    for (auto& wk : workers) wk->res.t0 = wk->res.t1 = -1.0;
    std::vector<double> tr_e0(kmax + 2, -1.0), tr_e1(kmax + 2, -1.0);
    for (int k = kfirst; k <= klast; ++k) {
        // keep P evaluations in flight: records of step k_dispatch-1, applied in order
        while (k_dispatch <= klast && k_dispatch < k + W) {
            lap(t_wait);
            err = tk_decomp_records(dc, k_dispatch, k_dispatch + 1, rec.data());
            lap(t_rec);
            if (!err) err = issue_upto(k_dispatch + depth);
            if (!err) err = ahead();
            lap(t_issue);
            if (err) break;
            apply_record(sv, k_dispatch - 1, rec.data());
            t_disp[k_dispatch] = clk::now();
            if (etr) tr_rec[k_dispatch] = since(t_disp[k_dispatch]);
            if (!split || sh.owner(k_dispatch)) {
                // owned iterations round-robin over the workers: at most P of them lie in a
                // window of W = P * NR, so a worker's previous one has been consumed
                const int w = nsub++ % P;
                wmap[k_dispatch] = w;
                submit(w, k_dispatch);
            }
            ++k_dispatch;
            lap(t_apply);
        }
        if (err) break;
        if (k_dispatch > klast) {
            err = read_gram();
            if (err) break;
        }
        IterResult other;
        IterResult* rp = &other;
        if (wmap[k] >= 0) {
            wait_done(wmap[k], k);
            rp = &workers[wmap[k]]->res;
        } else {
            err = mail_take(sv, k, other, t_disp[k]);
            if (err) break;
        }
        lap(t_wait);
        IterResult& r = *rp;
        {
            double* q = &sv->results[(size_t)(k - 1) * RES_N];
            q[RES_RC] = r.r_comp;
            q[RES_RN] = r.r_norm;
            q[RES_REL] = r.rel;
            q[RES_ORTH] = r.orth;
            q[RES_ST] = r.status;
            q[RES_US] = (wmap[k] >= 0 && r.t0 >= 0) ? 1e6 * (r.t1 - r.t0) : -1.0;
        }
        if (etr) {
            tr_cons[k] = since(clk::now());
            tr_e0[k] = r.t0 >= 0 ? std::chrono::duration<double, std::micro>(std::chrono::duration<double>(r.t0)).count() : -1;
            tr_e1[k] = r.t1 >= 0 ? std::chrono::duration<double, std::micro>(std::chrono::duration<double>(r.t1)).count() : -1;
        }
        if (r.status == TK_ERR_STATE) {
            err = tk_fail_internal(TK_ERR_STATE, "compressed solve failed (eigen / expm)");
            break;
        }
        if (r.status == TK_BREAKDOWN) {                       // CompressedNormBreakdown (:85-96)
            projres[k - 1] = r.r_comp;
            *outcome = 2;
            *k_end = k - 1;
            break;
        }
        relres[k - 1] = r.rel;
        projres[k - 1] = r.r_comp;
        orth[k - 1] = r.orth;
        if (r.rel < tol) {                                    // convergence (:108-118)
            *outcome = 1;
            *k_end = k;
            std::swap(sv->last, r);
            break;
        }
        if (k == klast) std::swap(sv->last, r);
    }
    const auto t_loop_end = clk::now();
    if (hp) hp->set_hot(false);
    if (!err && !gram_loss.empty())
        for (int k = kfirst; k <= std::min(*k_end, gram_k); ++k) orth[k - 1] = gram_loss[k - 1];
    quiesce();
    // converged on an iteration another rank evaluated: its y (lambda, Y) is needed here too
    // (basis_tensor_mul! of this rank's factors) -- evaluate it locally, bitwise the owner's
    if (!err && *outcome == 1 && sv->last.Y.empty()) evaluate(sv, *k_end, sv->last, sv->ws);
    const auto t_quiet = clk::now();
    if (etr) {
        if (FILE* f = fopen(etr, "w")) {
            fprintf(f, "# entry_to_loop_us=%.1f loop_us=%.1f quiesce_us=%.1f\n",
                    std::chrono::duration<double, std::micro>(t_begin - t_entry).count(), since(t_loop_end),
                    std::chrono::duration<double, std::micro>(t_quiet - t_loop_end).count());
            fprintf(f, "k,record_us,eval_start_us,eval_end_us,consumed_us\n");
            const double base = std::chrono::duration<double>(t_begin.time_since_epoch()).count();
            for (int k = kfirst; k <= *k_end; ++k)
                fprintf(f, "%d,%.1f,%.1f,%.1f,%.1f\n", k, tr_rec[k], tr_e0[k] >= 0 ? tr_e0[k] - 1e6 * base : -1.0,
                        tr_e1[k] >= 0 ? tr_e1[k] - 1e6 * base : -1.0, tr_cons[k]);
            fclose(f);
        }
    }
    if (stats)
        fprintf(stderr, "tk_solver_run: %d iterations, %d threads, %.1f us total: records %.1f, issue %.1f, "
                        "apply+submit %.1f, wait results %.1f (us per iteration)\n",
                *k_end - kfirst + 1, P,
                std::chrono::duration<double, std::micro>(clk::now() - t_begin).count(),
                t_rec / std::max(1, *k_end - kfirst + 1), t_issue / std::max(1, *k_end - kfirst + 1),
                t_apply / std::max(1, *k_end - kfirst + 1), t_wait / std::max(1, *k_end - kfirst + 1));
    return err;
    TK_API_END
}

}  // extern "C"
