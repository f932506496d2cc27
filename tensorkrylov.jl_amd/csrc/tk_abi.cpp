// tk_abi.cpp -- C ABI of libtkhip.so (include/tk.h): device state ownership, step
// sequencing (the per-factor fan-out of src/orthogonal_bases.jl:142-180 as ONE batched
// launch set over all of this rank's factors), the one RCCL all-reduce per step, and
// HIP-event timing.  No host pointer is retained after a call returns.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <rccl/rccl.h>

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <exception>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tk.h"
#include "tk_internal.h"
#include "tk_xsched.h"

// host polls of device-written words in host-mapped memory: TK_POLL_PAUSE=1 issues a pause
// between reads (fewer reads of lines the GPU is writing over the fabric)
#ifndef TK_POLL_PAUSE
#define TK_POLL_PAUSE 1
#endif
#if TK_POLL_PAUSE
#define TK_POLL_RELAX() _mm_pause()
#else
#define TK_POLL_RELAX() do { } while (0)
#endif

using namespace tk;

// Test build (tests/_build/libtkhip_test.so: -DTK_TEST_BUILD=1, made by __graft_entry__.build()
// for the test suite only).  The switches that skip work, drop guards or inject failures
// (TKHIP_TEST_SKIP, _XCH_SKIP, _NO_GUARD, _SHARED_XSIG, _XCH_STALL, _FAIL_STEP, _FUSE_SPIN)
// and the multi-process transport on one GPU (tk_comm_init_test) exist only there: in the
// product library TEST_ENV is a constant NULL, so no environment variable can make
// libtkhip.so produce wrong records.
#ifndef TK_TEST_BUILD
#define TK_TEST_BUILD 0
#endif
#if TK_TEST_BUILD
#define TEST_ENV(name) getenv(name)
#else
#define TEST_ENV(name) ((const char*)nullptr)
#endif

// ------------------------------------------------------------------ host issue profile
// TKHIP_HOST_PROFILE=1 (diagnostics): host time spent in each part of a step's issue, summed
// over the process and printed to stderr at exit -- where the 8-15 us per step of
// tk_decomp_step go (launches, exchange calls, event queries, the rest)
enum { HP_STEP = 0, HP_D1, HP_RED, HP_GUARD, HP_XCH, HP_NCCL, HP_MIRROR, HP_BK, HP_GQ, HP_N };
static const char* const hp_name[HP_N] = {"tk_decomp_step (all)", "k_arn_d1 launch", "k_reduce256 launch",
                                          "slot guard", "exchange_range (all)", "ncclAllReduce",
                                          "mirror launch", "bk/complete/xsched", "slot guard: event query"};
struct HostProf {
    bool on = false;
    double us[HP_N] = {};
    long n[HP_N] = {};
    HostProf() {
        const char* e = getenv("TKHIP_HOST_PROFILE");
        on = e && e[0] == '1';
    }
    ~HostProf() {
        if (!on || !n[HP_STEP]) return;
        fprintf(stderr, "[tkhip host profile] %ld steps\n", n[HP_STEP]);
        for (int i = 0; i < HP_N; ++i)
            if (n[i])
                fprintf(stderr, "  %-24s %8ld calls %9.2f us/call %7.2f us/step\n", hp_name[i], n[i], us[i] / n[i],
                        us[i] / n[HP_STEP]);
    }
};
static HostProf g_hp;
struct HpScope {
    int i;
    std::chrono::steady_clock::time_point t0;
    explicit HpScope(int i_) : i(g_hp.on ? i_ : -1) {
        if (i >= 0) t0 = std::chrono::steady_clock::now();
    }
    ~HpScope() {
        if (i < 0) return;
        g_hp.us[i] += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        ++g_hp.n[i];
    }
};

// ------------------------------------------------------------------ errors
// a fixed buffer: recording an error never allocates (a bad_alloc is itself reported here)
static thread_local char g_err[1024];

static tk_status fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

// tk_host.cpp reports through the same thread-local message
tk_status tk_fail_internal(int code, const char* msg) { return fail(code, "%s", msg); }

// Every exported body runs inside TK_API_BEGIN / TK_API_END: host containers (std::vector)
// may throw, and tk.h promises that nothing throws across the ABI.
#define TK_API_BEGIN try {
#define TK_API_END                                                                        \
    }                                                                                     \
    catch (const std::bad_alloc&) { return fail(TK_ERR_ALLOC, "host allocation failed"); } \
    catch (const std::exception& ex_) { return fail(TK_ERR_INTERNAL, "%s", ex_.what()); } \
    catch (...) { return fail(TK_ERR_INTERNAL, "unknown C++ exception"); }

#define HIPCHK(x)                                                                         \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) return fail(TK_ERR_HIP, "%s: %s", #x, hipGetErrorString(e_)); \
    } while (0)
#define LAUNCHCHK(what)                                                                   \
    do {                                                                                  \
        hipError_t e_ = hipGetLastError();                                                \
        if (e_ != hipSuccess) return fail(TK_ERR_HIP, "launch %s: %s", what, hipGetErrorString(e_)); \
    } while (0)
#define NCCLCHK(x)                                                                        \
    do {                                                                                  \
        ncclResult_t r_ = (x);                                                            \
        if (r_ != ncclSuccess) return fail(TK_ERR_RCCL, "%s: %s", #x, ncclGetErrorString(r_)); \
    } while (0)
#define CHECKARG(c, msg)                      \
    do {                                      \
        if (!(c)) return fail(TK_ERR_ARG, "%s", msg); \
    } while (0)

// ------------------------------------------------------------------ context
enum { TCLS_STEP = 0, TCLS_PASS1 = 1, TCLS_PASS2 = 2, TCLS_FIN = 3, TCLS_RED = 4, TCLS_VY = 5, TCLS_XCH = 6,
       TCLS_SWEEP = 7, TCLS_GRAM = 8, TCLS_N = 9 };

struct tk_ctx {
    int device = 0;
    hipStream_t stream = nullptr;    // compute
    hipStream_t xstream = nullptr;   // per-step record exchange (RCCL), overlaps compute
    hipStream_t gstream = nullptr;   // deferred orthogonality Gram (tk_decomp_gram), overlaps compute
    hipStream_t fstream = nullptr;   // the second factor group of one-sweep Arnoldi steps (tk_decomp)
    ncclComm_t comm = nullptr;
    struct TestComm* tcomm = nullptr;   // test build: the shared-memory stand-in for RCCL
    int nranks = 1, rank = 0;
    int timing = 0;   // 0 off, 1 step level, 2 per kernel class
    std::vector<hipEvent_t> ev[TCLS_N];   // start/stop pairs
    double ms[TCLS_N] = {0};
    long cnt[TCLS_N] = {0};
    double* xbuf = nullptr;   // host-allreduce staging
    size_t xcap = 0;
    // a wait on the other ranks expired (TKHIP_WAIT_S): a collective may still be running on
    // this device, so its buffers, streams and communicator are left to process exit
    bool stuck = false;
    std::vector<hipEvent_t> evpool;   // recycled timing events (no hipEventCreate per step)
    // host-mapped error word of the fused one-sweep launches (k_arn_d1's bounded wait for its
    // in-launch reducers gave up: that step's values are wrong).  Sticky; every call that
    // hands results out after a device sync checks it (werr_check)
    unsigned int* werr = nullptr;
    // Handles may be destroyed in any order (Julia finalizers, Python GC): matrices and
    // decompositions hold a reference on their context, decompositions on their matrices.
    std::atomic<int> refs{1};
};

struct Timer {
    tk_ctx* c;
    int cls;
    bool on;
    hipStream_t st;
    hipEvent_t b = nullptr;
    Timer(tk_ctx* c_, int cls_, int level, hipStream_t s_ = nullptr)
        : c(c_), cls(cls_), on(c_->timing >= level), st(s_ ? s_ : c_->stream) {
        if (!on) return;
        hipEvent_t a;
        if (!take(a) || !take(b)) { on = false; return; }
        hipEventRecord(a, st);
        c->ev[cls].push_back(a);
    }
    bool take(hipEvent_t& e) {
        if (!c->evpool.empty()) {
            e = c->evpool.back();
            c->evpool.pop_back();
            return true;
        }
        // timing only: no system-scope fence on record (with it every record cost ~10 us of
        // GPU idle time -- a cache writeback -- between the kernels it brackets)
        return hipEventCreateWithFlags(&e, hipEventDisableSystemFence) == hipSuccess;
    }
    ~Timer() {
        if (!on) return;
        hipEventRecord(b, st);
        c->ev[cls].push_back(b);
    }
};

static void drain_timers(tk_ctx* c) {
    for (int k = 0; k < TCLS_N; ++k) {
        auto& v = c->ev[k];
        if (v.empty()) continue;
        hipEventSynchronize(v.back());
        for (size_t i = 0; i + 1 < v.size(); i += 2) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, v[i], v[i + 1]) == hipSuccess) {
                c->ms[k] += ms;
                c->cnt[k] += 1;
            }
            c->evpool.push_back(v[i]);
            c->evpool.push_back(v[i + 1]);
        }
        v.clear();
    }
}

// ------------------------------------------------------------------ bounded waits
// Every wait that can depend on another rank (the records exchange, host all-reduces, a
// stream that may sit behind a collective) has a wall-clock limit: TKHIP_WAIT_S seconds
// (default 120).  On expiry the call returns TK_ERR_RCCL saying what it waited for, which
// record slot and step, and RCCL's asynchronous error state -- a peer that never joins a
// collective ends in a diagnosis, not in a job killed at its time limit.
static double wait_limit_s() {
    const char* e = getenv("TKHIP_WAIT_S");
    const double v = e ? atof(e) : 120.0;
    return v > 0 ? v : 120.0;
}

// a multi-rank communicator: RCCL, or (test build) the shared-memory stand-in
static inline bool has_peers(const tk_ctx* c) { return c->comm != nullptr || c->tcomm != nullptr; }

static const char* comm_state(tk_ctx* c) {
    if (c->tcomm) return "test transport: a peer has not posted its contribution";
    if (!c->comm) return "no communicator";
    ncclResult_t r = ncclSuccess;
    if (ncclCommGetAsyncError(c->comm, &r) != ncclSuccess) return "ncclCommGetAsyncError failed";
    return r == ncclSuccess ? "no asynchronous error: a peer has not entered the collective" : ncclGetErrorString(r);
}

static tk_status wait_expired(tk_ctx* c, const char* what, int slot) {
    c->stuck = true;
    return fail(TK_ERR_RCCL, "%s: not complete after %.0f s (record slot %d = step %d; rank %d of %d; RCCL: %s)",
                what, wait_limit_s(), slot, slot - 1, c->rank, c->nranks, comm_state(c));
}

// Without a communicator (one GPU) waits are plain synchronisations: queued work of any
// length is waited for and the context is never marked stuck.  TKHIP_LOCAL_WAIT_S > 0 bounds
// them too (a device hang then returns TK_ERR_HIP naming the wait instead of blocking the
// host; the context stays usable) -- off by default: a long legitimate queue must not fail
static double local_limit_s() {
    static const double v = [] {
        const char* e = getenv("TKHIP_LOCAL_WAIT_S");
        const double x = e ? atof(e) : 0.0;
        return x > 0 ? x : 0.0;
    }();
    return v;
}
// the limit a wait of this context has: TKHIP_WAIT_S with peers, else TKHIP_LOCAL_WAIT_S (0: none)
static double ctx_wait_limit(const tk_ctx* c) { return has_peers(c) ? wait_limit_s() : local_limit_s(); }

struct Deadline {
    typedef std::chrono::steady_clock clk;
    clk::time_point t0 = clk::now();
    double lim = wait_limit_s();
    Deadline() = default;
    explicit Deadline(double l) : lim(l) {}
    // (lim 0: never expires)
    bool over() const { return lim > 0 && elapsed() > lim; }
    double elapsed() const { return std::chrono::duration<double>(clk::now() - t0).count(); }
    // true once expired; backs off to short sleeps after the first millisecond
    bool tick() {
        const double el = elapsed();
        if (el > lim) return true;
        if (el > 1e-3) std::this_thread::sleep_for(std::chrono::microseconds(20));
        return false;
    }
};

// hipStreamSynchronize with a deadline -- only where another rank can be involved: without a
// communicator (one GPU) queued work of any length is waited for plainly, and never marks the
// context stuck
static tk_status local_expired(const char* what, double lim) {
    return fail(TK_ERR_HIP, "%s: device work not complete after %.0f s (TKHIP_LOCAL_WAIT_S)", what, lim);
}

static tk_status sync_bounded(tk_ctx* c, hipStream_t s, const char* what, int slot = -1) {
    if (!has_peers(c) && local_limit_s() <= 0) {
        const hipError_t e = hipStreamSynchronize(s);
        return e == hipSuccess ? TK_OK : fail(TK_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    }
    Deadline dl(ctx_wait_limit(c));
    for (;;) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) return TK_OK;
        if (e != hipErrorNotReady) return fail(TK_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
        if (dl.tick()) return has_peers(c) ? wait_expired(c, what, slot) : local_expired(what, dl.lim);
    }
}

// hipEventSynchronize with a deadline
static tk_status event_bounded(tk_ctx* c, hipEvent_t ev, const char* what, int slot = -1) {
    if (!has_peers(c) && local_limit_s() <= 0) {
        const hipError_t e = hipEventSynchronize(ev);
        return e == hipSuccess ? TK_OK : fail(TK_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    }
    Deadline dl(ctx_wait_limit(c));
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return TK_OK;
        if (e != hipErrorNotReady) return fail(TK_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
        if (dl.tick()) return has_peers(c) ? wait_expired(c, what, slot) : local_expired(what, dl.lim);
    }
}

// A fused one-sweep launch's wait for its in-launch reducers gave up (the context's error
// word, set by the device): results handed out after that are wrong.  Checked after every
// device-completion point that hands results to the caller
static tk_status werr_check(const tk_ctx* c, const char* what) {
    if (c->werr && __atomic_load_n(c->werr, __ATOMIC_ACQUIRE))
        return fail(TK_ERR_INTERNAL, "%s: a fused one-sweep launch's wait for its reducers gave up, so the "
                                     "records of that step are wrong (TKHIP_D1_FUSE=0 avoids the fused launch)", what);
    return TK_OK;
}

#define STUCKCHK(c)                                                                                   \
    do {                                                                                              \
        if ((c)->stuck)                                                                               \
            return fail(TK_ERR_RCCL, "the communicator is unusable: an earlier wait on the other ranks " \
                                     "expired (TKHIP_WAIT_S)");                                       \
    } while (0)


// ------------------------------------------------------------------ test transport
// Several processes on ONE GPU cannot form an RCCL communicator (RCCL refuses: "Duplicate GPU
// detected"), so the multi-rank exchange -- factor groups under an exchange, per-factor signal
// words, alternating send buffers, coalesced slot guards, the evaluation mailbox, replicas --
// is exercised with real peer processes through this stand-in for ncclAllReduce (test build
// only).  Node-local POSIX shared memory /dev/shm/tkhip_tc_<key> holds, per rank, two buffers
// (by collective sequence parity), a posted word per buffer and a consumed word.  Collective
// number s: wait until every rank has consumed s-2 (the buffer's last use), copy this rank's
// contribution in, post s, wait for every rank's post of s, combine in rank order (sum or
// max: the records exchange adds zeros to each row, so the sum is exact), consume s.  The
// records exchange stays stream-ordered on the exchange stream: send rows -> host-mapped
// coherent memory, the combine in a host function (hipLaunchHostFunc), result -> the receive
// buffer.  The two copies are k_mirror_records launches (device-side loads through L2,
// system-scope stores), not hipMemcpyAsync: a DMA engine reads HBM behind the L2, where a
// LanczosReorth step's records -- released at device scope only (its exchange waits on an
// event without a system fence) -- are not yet written back.  Every rank issues the same
// collectives in the same order (tk_xsched.h), so the
// sequence numbers agree.  Host all-reduces (preflight, agreements) wait for the exchange
// stream first and combine on the host directly.  Every wait is bounded by TKHIP_WAIT_S.
#if TK_TEST_BUILD
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
struct TcRank {
    std::atomic<unsigned long long> posted[2];
    std::atomic<unsigned long long> consumed;
    char pad[40];
};
struct TcHdr {
    std::atomic<unsigned long long> attached;
    unsigned long long nranks, cap, magic;
    char pad[32];
};
static_assert(sizeof(TcRank) == 64 && sizeof(TcHdr) == 64, "shared-memory layout");
struct TestComm {
    TcHdr* hdr = nullptr;
    size_t bytes = 0;
    int nranks = 1, rank = 0;
    size_t cap = 0;                     // doubles per buffer
    unsigned long long seq = 0;         // collectives issued by this process
    double* hsend = nullptr;            // host-mapped staging of the records exchange
    double* hrecv = nullptr;
    size_t hcap = 0;
    unsigned long long* hword = nullptr;   // (the copy kernels' done word: unused)
    std::atomic<int> failed{0};         // a wait expired inside a host function
    TcRank* rk(int q) const {
        return (TcRank*)((char*)hdr + sizeof(TcHdr) + (size_t)q * (sizeof(TcRank) + 2 * cap * sizeof(double)));
    }
    double* buf(int q, int p) const { return (double*)(rk(q) + 1) + (size_t)p * cap; }
};
static const unsigned long long TC_MAGIC = 0x746b68697074636dull;

// one chunk (n <= cap) of collective number s; false when a wait expired (out is NaN then)
static bool tc_chunk(TestComm* tc, const double* in, double* out, size_t n, bool mx, unsigned long long s) {
    const int p = (int)(s & 1);
    Deadline dl(wait_limit_s());
    auto wait_all = [&](auto pred) {
        for (int q = 0; q < tc->nranks; ++q)
            while (!pred(tc->rk(q)))
                if (dl.tick()) return false;
        return true;
    };
    bool ok = s <= 2 || wait_all([&](TcRank* r) { return r->consumed.load(std::memory_order_acquire) >= s - 2; });
    TcRank* me = tc->rk(tc->rank);
    if (ok) {
        memcpy(tc->buf(tc->rank, p), in, n * sizeof(double));
        me->posted[p].store(s, std::memory_order_release);
        ok = wait_all([&](TcRank* r) { return r->posted[p].load(std::memory_order_acquire) >= s; });
    }
    if (!ok) {
        for (size_t i = 0; i < n; ++i) out[i] = NAN;
        tc->failed.store(1);
        return false;
    }
    for (size_t i = 0; i < n; ++i) {
        double a = tc->buf(0, p)[i];
        for (int q = 1; q < tc->nranks; ++q) {
            const double b = tc->buf(q, p)[i];
            a = mx ? (b > a ? b : a) : a + b;
        }
        out[i] = a;
    }
    me->consumed.store(s, std::memory_order_release);
    return true;
}
// a collective over any count: ceil(count / cap) sequence numbers from seq0
static bool tc_run(TestComm* tc, const double* in, double* out, size_t count, bool mx, unsigned long long seq0) {
    bool ok = true;
    for (size_t off = 0, k = 0; off < count || (count == 0 && k == 0); off += tc->cap, ++k) {
        const size_t n = std::min(tc->cap, count - off);
        ok = tc_chunk(tc, in + off, out + off, n, mx, seq0 + k) && ok;
        if (count == 0) break;
    }
    return ok;
}
static unsigned long long tc_nseq(const TestComm* tc, size_t count) {
    return count == 0 ? 1 : (count + tc->cap - 1) / tc->cap;
}
static tk_status tc_allreduce(tk_ctx* c, const double* in, double* out, size_t count, bool mx, const char* what) {
    TestComm* tc = c->tcomm;
    const unsigned long long s0 = tc->seq + 1;
    tc->seq += tc_nseq(tc, count);
    if (tc->failed.load() || !tc_run(tc, in, out, count, mx, s0)) return wait_expired(c, what, -1);
    return TK_OK;
}
struct TcJob {
    TestComm* tc;
    size_t n;
    unsigned long long s0;
};
static void tc_job_cb(void* arg) {
    TcJob* jb = (TcJob*)arg;
    if (!jb->tc->failed.load()) tc_run(jb->tc, jb->tc->hsend, jb->tc->hrecv, jb->n, false, jb->s0);
    delete jb;
}
static tk_status tc_exchange(tk_ctx* c, const double* s, double* r, size_t tot, hipStream_t st) {
    TestComm* tc = c->tcomm;
    if (tc->failed.load()) return wait_expired(c, "records exchange (test transport)", -1);
    const unsigned flags = hipHostMallocMapped | hipHostMallocCoherent;
    if (!tc->hword) HIPCHK(hipHostMalloc((void**)&tc->hword, 64, flags));
    if (tot > tc->hcap) {
        tk_status sb = sync_bounded(c, st, "test transport staging");
        if (sb) return sb;
        if (tc->hsend) hipHostFree(tc->hsend);
        if (tc->hrecv) hipHostFree(tc->hrecv);
        tc->hsend = tc->hrecv = nullptr;
        tc->hcap = 0;
        HIPCHK(hipHostMalloc((void**)&tc->hsend, tot * sizeof(double), flags));
        HIPCHK(hipHostMalloc((void**)&tc->hrecv, tot * sizeof(double), flags));
        tc->hcap = tot;
    }
    TcJob* jb = new TcJob{tc, tot, tc->seq + 1};
    tc->seq += tc_nseq(tc, tot);
    launch_mirror_records(s, tc->hsend, (int)tot, tc->hword, 1, tc->seq, st);
    LAUNCHCHK("test transport: send rows to the host");
    hipError_t e = hipLaunchHostFunc(st, tc_job_cb, jb);
    if (e != hipSuccess) {
        delete jb;
        return fail(TK_ERR_HIP, "hipLaunchHostFunc: %s", hipGetErrorString(e));
    }
    launch_mirror_records(tc->hrecv, r, (int)tot, tc->hword, 1, tc->seq, st);
    LAUNCHCHK("test transport: combined rows to the device");
    return TK_OK;
}
static void tc_destroy(tk_ctx* c) {
    TestComm* tc = c->tcomm;
    if (!tc) return;
    if (tc->hsend) hipHostFree(tc->hsend);
    if (tc->hrecv) hipHostFree(tc->hrecv);
    if (tc->hword) hipHostFree(tc->hword);
    if (tc->hdr) munmap(tc->hdr, tc->bytes);
    delete tc;
    c->tcomm = nullptr;
}
extern "C" tk_status tk_comm_init_test(tk_ctx* c, const char* key, int nranks, int rank) { TK_API_BEGIN
    CHECKARG(c && key && nranks >= 1 && rank >= 0 && rank < nranks, "bad argument");
    CHECKARG(!c->comm && !c->tcomm, "the context already has a communicator");
    for (const char* q = key; *q; ++q)
        CHECKARG((*q >= '0' && *q <= '9') || (*q >= 'a' && *q <= 'z') || (*q >= 'A' && *q <= 'Z') || *q == '_',
                 "key must be [0-9A-Za-z_]");
    char name[200];
    snprintf(name, sizeof name, "/dev/shm/tkhip_tc_%s", key);
    const size_t cap = 1 << 16;
    const size_t bytes = sizeof(TcHdr) + (size_t)nranks * (sizeof(TcRank) + 2 * cap * sizeof(double));
    Deadline dl(wait_limit_s());
    TcHdr* h = nullptr;
    if (rank == 0) {
        char tmp[220];
        snprintf(tmp, sizeof tmp, "%s.%d.tmp", name, (int)getpid());
        int fd = open(tmp, O_RDWR | O_CREAT | O_EXCL, 0600);
        if (fd < 0 || ftruncate(fd, (off_t)bytes) != 0) {
            if (fd >= 0) close(fd), unlink(tmp);
            return fail(TK_ERR_STATE, "tk_comm_init_test: cannot create %s", tmp);
        }
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        close(fd);
        if (m == MAP_FAILED) {
            unlink(tmp);
            return fail(TK_ERR_STATE, "tk_comm_init_test: mmap failed");
        }
        memset(m, 0, bytes);
        h = (TcHdr*)m;
        h->nranks = (unsigned long long)nranks;
        h->cap = cap;
        h->magic = TC_MAGIC;
        h->attached.store(1, std::memory_order_release);
        if (rename(tmp, name) != 0) {
            munmap(m, bytes);
            unlink(tmp);
            return fail(TK_ERR_STATE, "tk_comm_init_test: cannot publish %s", name);
        }
        while (h->attached.load(std::memory_order_acquire) < (unsigned long long)nranks)
            if (dl.tick()) {
                unlink(name);
                munmap(m, bytes);
                return fail(TK_ERR_RCCL, "tk_comm_init_test: only %llu of %d ranks attached", h->attached.load(), nranks);
            }
        unlink(name);   // every rank holds its mapping: nothing is left in /dev/shm
    } else {
        int fd;
        while ((fd = open(name, O_RDWR)) < 0)
            if (dl.tick()) return fail(TK_ERR_RCCL, "tk_comm_init_test: rank 0 never published %s", name);
        struct stat sb;
        void* m = (fstat(fd, &sb) == 0 && (size_t)sb.st_size == bytes)
                      ? mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0) : MAP_FAILED;
        close(fd);
        h = (TcHdr*)m;
        if (m == MAP_FAILED || h->magic != TC_MAGIC || h->nranks != (unsigned long long)nranks || h->cap != cap) {
            if (m != MAP_FAILED) munmap(m, bytes);
            return fail(TK_ERR_STATE, "tk_comm_init_test: %s does not describe this job", name);
        }
        h->attached.fetch_add(1, std::memory_order_acq_rel);
    }
    TestComm* tc = new TestComm();
    tc->hdr = h;
    tc->bytes = bytes;
    tc->nranks = nranks;
    tc->rank = rank;
    tc->cap = cap;
    c->tcomm = tc;
    c->nranks = nranks;
    c->rank = rank;
    return TK_OK;
    TK_API_END
}
#else
struct TestComm {};
static tk_status tc_allreduce(tk_ctx*, const double*, double*, size_t, bool, const char*) { return TK_ERR_INTERNAL; }
static tk_status tc_exchange(tk_ctx*, const double*, double*, size_t, hipStream_t) { return TK_ERR_INTERNAL; }
static void tc_destroy(tk_ctx*) {}
#endif

extern "C" {

const char* tk_last_error(void) { return g_err; }
int tk_version(void) { return 100; }

tk_status tk_ctx_create(int device, tk_ctx** out) { TK_API_BEGIN
    CHECKARG(out, "out is NULL");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(TK_ERR_NODEV, "no HIP device visible");
    CHECKARG(device >= 0 && device < ndev, "device ordinal out of range");
    HIPCHK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(TK_ERR_NODEV, "device %d is %s; libtkhip is built for gfx950 only", device, prop.gcnArchName);
    tk_ctx* c = new tk_ctx();
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->xstream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->gstream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->fstream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return fail(TK_ERR_HIP, "hipStreamCreate: %s", hipGetErrorString(e));
    }
    {
        void* hp = nullptr;
        if (hipHostMalloc(&hp, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
            hipStreamDestroy(c->stream);
            hipStreamDestroy(c->xstream);
            hipStreamDestroy(c->gstream);
            hipStreamDestroy(c->fstream);
            delete c;
            return fail(TK_ERR_ALLOC, "tk_ctx_create: error word");
        }
        c->werr = (unsigned int*)hp;
        *c->werr = 0;
    }
    *out = c;
    return TK_OK;
    TK_API_END
}


static void ctx_release(tk_ctx* c) {
    if (--c->refs > 0) return;
    hipSetDevice(c->device);
    if (!c->stuck) sync_bounded(c, c->stream, "tk_ctx_destroy");
    if (!c->stuck) sync_bounded(c, c->xstream, "tk_ctx_destroy");
    if (!c->stuck) sync_bounded(c, c->gstream, "tk_ctx_destroy");
    if (!c->stuck) sync_bounded(c, c->fstream, "tk_ctx_destroy");
    if (c->stuck) return;   // a collective may still run: its resources are left to process exit
    drain_timers(c);
    for (hipEvent_t e : c->evpool) hipEventDestroy(e);
    if (c->comm) ncclCommDestroy(c->comm);
    tc_destroy(c);
    if (c->xbuf) hipFree(c->xbuf);
    if (c->werr) hipHostFree(c->werr);
    hipStreamDestroy(c->stream);
    hipStreamDestroy(c->xstream);
    hipStreamDestroy(c->gstream);
    hipStreamDestroy(c->fstream);
    delete c;
}

tk_status tk_ctx_destroy(tk_ctx* c) { TK_API_BEGIN
    if (!c) return TK_OK;
    ctx_release(c);
    return TK_OK;
    TK_API_END
}

tk_status tk_ctx_sync(tk_ctx* c) { TK_API_BEGIN
    CHECKARG(c, "ctx is NULL");
    HIPCHK(hipSetDevice(c->device));
    STUCKCHK(c);
    tk_status st = sync_bounded(c, c->stream, "tk_ctx_sync (compute stream)");
    if (st == TK_OK) st = sync_bounded(c, c->gstream, "tk_ctx_sync (Gram stream)");
    if (st == TK_OK) st = sync_bounded(c, c->fstream, "tk_ctx_sync (factor-group stream)");
    if (st == TK_OK) st = sync_bounded(c, c->xstream, "tk_ctx_sync (exchange stream)");
    return st ? st : werr_check(c, "tk_ctx_sync");
    TK_API_END
}

tk_status tk_comm_unique_id(char id_out[128]) { TK_API_BEGIN
    CHECKARG(id_out, "id_out is NULL");
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");
    memcpy(id_out, &id, 128);
    return TK_OK;
    TK_API_END
}

tk_status tk_comm_init(tk_ctx* c, const char id[128], int nranks, int rank) { TK_API_BEGIN
    CHECKARG(c && id, "NULL argument");
    CHECKARG(nranks >= 1 && rank >= 0 && rank < nranks, "bad nranks/rank");
    HIPCHK(hipSetDevice(c->device));
    ncclUniqueId uid;
    memcpy(&uid, id, 128);
    NCCLCHK(ncclCommInitRank(&c->comm, nranks, uid, rank));
    c->nranks = nranks;
    c->rank = rank;
    return TK_OK;
    TK_API_END
}

// In-place all-reduce of host doubles through the device, after every records exchange
// already enqueued (collectives keep one order on every rank); bounded waits.
static tk_status host_allreduce(tk_ctx* c, double* buf, size_t count, ncclRedOp_t op, const char* what) {
    STUCKCHK(c);
    HIPCHK(hipSetDevice(c->device));
    if (count > c->xcap) {
        if (c->xbuf) hipFree(c->xbuf);
        c->xbuf = nullptr;
        HIPCHK(hipMalloc(&c->xbuf, count * sizeof(double)));
        c->xcap = count;
    }
    tk_status st = sync_bounded(c, c->xstream, what);
    if (st) return st;
    if (c->tcomm) return tc_allreduce(c, buf, buf, count, op == ncclMax, what);   // (host memory already)
    HIPCHK(hipMemcpyAsync(c->xbuf, buf, count * sizeof(double), hipMemcpyHostToDevice, c->stream));
    NCCLCHK(ncclAllReduce(c->xbuf, c->xbuf, count, ncclDouble, op, c->comm, c->stream));
    HIPCHK(hipMemcpyAsync(buf, c->xbuf, count * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    return sync_bounded(c, c->stream, what);
}

tk_status tk_comm_allreduce_host(tk_ctx* c, double* buf, size_t count) { TK_API_BEGIN
    CHECKARG(c && buf, "NULL argument");
    if (!has_peers(c) || c->nranks == 1) return TK_OK;
    return host_allreduce(c, buf, count, ncclSum, "tk_comm_allreduce_host");
    TK_API_END
}

tk_status tk_comm_count(tk_ctx* c, int* nranks_out) { TK_API_BEGIN
    CHECKARG(c && nranks_out, "NULL argument");
    *nranks_out = 0;
    if (c->tcomm) *nranks_out = c->nranks;
    if (!c->comm) return TK_OK;
    int n = 0;
    NCCLCHK(ncclCommCount(c->comm, &n));
    *nranks_out = n;
    return TK_OK;
    TK_API_END
}

// ------------------------------------------------------------------ matrices
struct tk_mat {
    tk_ctx* ctx;
    std::atomic<int> refs{1};
    int64_t n = 0, nnz = 0;
    int* rowptr = nullptr;
    int* col = nullptr;
    double* val = nullptr;
    int* doff = nullptr;
    double* dval = nullptr;
    int ndiag = 0;
    int64_t dld = 0;
    double* dconst = nullptr;
    int toep = 0;
    int hl = 0, hu = 0;   // lower / upper bandwidth of the DIA storage
    long long* sptr = nullptr;
    int* swidth = nullptr;
    int* rowlen = nullptr;
    int* scol = nullptr;
    double* sval = nullptr;
    int sell = 0;
    SpM spm() const {
        SpM m;
        m.rowptr = rowptr;
        m.col = col;
        m.val = val;
        m.doff = doff;
        m.dval = dval;
        m.ndiag = ndiag;
        m.dld = dld;
        m.dconst = dconst;
        m.toep = toep;
        m.sptr = sptr;
        m.swidth = swidth;
        m.rowlen = rowlen;
        m.scol = scol;
        m.sval = sval;
        m.sell = sell;
        m.n = n;
        return m;
    }
};

static void free_mat(tk_mat* A) {
    hipFree(A->rowptr);
    hipFree(A->col);
    hipFree(A->val);
    hipFree(A->doff);
    hipFree(A->dval);
    hipFree(A->dconst);
    hipFree(A->sptr);
    hipFree(A->swidth);
    hipFree(A->rowlen);
    hipFree(A->scol);
    hipFree(A->sval);
    delete A;
}

// DIA when the matrix is banded with at most TK_MAX_DIAG diagonals that are at least
// 3/4 full (Laplace: 3, ConvDiff: 4); TKHIP_FORCE_CSR=1 disables it.
#define TK_MAX_DIAG 8
static void build_dia(int64_t n, const std::vector<int>& rp, const std::vector<int>& ci,
                      const std::vector<double>& v, std::vector<int>& offs, std::vector<double>& dv,
                      int64_t& dld, std::vector<double>& dc, int& toep) {
    toep = 0;
    offs.clear();
    const char* env = getenv("TKHIP_FORCE_CSR");
    if (env && env[0] == '1') return;
    std::vector<int> seen;
    for (int64_t r = 0; r < n; ++r)
        for (int p = rp[r]; p < rp[r + 1]; ++p) {
            // a duplicate (row, column) entry of a non-canonical CSC: the scatter mul! adds
            // both products in turn, which CSR/SELL reproduce bitwise and one DIA slot cannot
            if (p > rp[r] && ci[p] == ci[p - 1]) return;
            const int o = ci[p] - (int)r;
            if (std::find(seen.begin(), seen.end(), o) == seen.end()) {
                seen.push_back(o);
                if ((int)seen.size() > TK_MAX_DIAG) return;
            }
        }
    std::sort(seen.begin(), seen.end());
    const int64_t nd = (int64_t)seen.size();
    if (nd == 0 || (int64_t)ci.size() * 4 < nd * n * 3) return;
    dld = (n + 255) / 256 * 256;
    // the device keeps at least 4 diagonal rows (zero rows, offset 0): the <= 4-diagonal
    // SpMV issues all its loads unconditionally
    dv.assign((size_t)std::max<int64_t>(nd, 4) * dld, 0.0);
    for (int64_t r = 0; r < n; ++r)
        for (int p = rp[r]; p < rp[r + 1]; ++p) {
            const int o = ci[p] - (int)r;
            const int q = (int)(std::lower_bound(seen.begin(), seen.end(), o) - seen.begin());
            dv[(size_t)q * dld + r] = v[p];
        }
    offs = seen;
    // Toeplitz band (the gallery's Laplace / ConvDiff): every in-range position of each
    // diagonal present with one bit-identical value -> the SpMV reads no matrix values
    std::vector<int64_t> count(nd, 0);
    for (int64_t r = 0; r < n; ++r)
        for (int p = rp[r]; p < rp[r + 1]; ++p)
            ++count[std::lower_bound(seen.begin(), seen.end(), ci[p] - (int)r) - seen.begin()];
    dc.assign(std::max<int64_t>(nd, 4), 0.0);
    bool tz = true;
    for (int64_t q = 0; q < nd && tz; ++q) {
        const int64_t o = seen[q];
        const int64_t r0 = std::max<int64_t>(0, -o), r1 = std::min<int64_t>(n, n - o);
        if (count[q] != r1 - r0) { tz = false; break; }
        const double c0 = dv[(size_t)q * dld + r0];
        for (int64_t r = r0; r < r1; ++r)
            if (memcmp(&dv[(size_t)q * dld + r], &c0, sizeof(double)) != 0) { tz = false; break; }
        dc[q] = c0;
    }
    toep = tz ? 1 : 0;
}
static int dia_rows(int ndiag) { return ndiag < 4 ? 4 : ndiag; }

// SELL-256 (sliced ELL, slice = 256-row tile) for matrices that are not banded, when the
// padding stays within 2x nnz; TKHIP_FORCE_CSR=1 disables it.
static bool build_sell(int64_t n, const std::vector<int>& rp, const std::vector<int>& ci,
                       const std::vector<double>& v, std::vector<long long>& sptr, std::vector<int>& sw,
                       std::vector<int>& rl, std::vector<int>& sc, std::vector<double>& sv) {
    const char* env = getenv("TKHIP_FORCE_CSR");
    if (env && env[0] == '1') return false;
    const int64_t nt = (n + 255) / 256;
    sptr.assign(nt, 0);
    sw.assign(nt, 0);
    rl.assign(nt * 256, 0);
    long long slots = 0;
    for (int64_t t = 0; t < nt; ++t) {
        int w = 0;
        for (int64_t r = t * 256; r < std::min<int64_t>(n, (t + 1) * 256); ++r) {
            rl[r] = rp[r + 1] - rp[r];
            w = std::max(w, rl[r]);
        }
        sptr[t] = slots;
        sw[t] = w;
        slots += (long long)w * 256;
    }
    if (slots > 2 * (long long)ci.size() + 256 || slots >= (long long)INT32_MAX) return false;
    sc.assign(slots, 0);
    sv.assign(slots, 0.0);
    for (int64_t t = 0; t < nt; ++t)
        for (int l = 0; l < 256; ++l) {
            const int64_t r = t * 256 + l;
            for (int q = 0; q < sw[t]; ++q) {
                const long long e = sptr[t] + (long long)q * 256 + l;
                if (r < n && q < rl[r]) {
                    sc[e] = ci[rp[r] + q];
                    sv[e] = v[rp[r] + q];
                } else {
                    sc[e] = (int)std::min<int64_t>(r, n - 1);
                }
            }
        }
    return true;
}

static tk_status upload_csr(tk_ctx* c, int64_t n, const std::vector<int>& rp, const std::vector<int>& ci,
                            const std::vector<double>& v, tk_mat** out) {
    tk_mat* A = new tk_mat();
    A->ctx = c;
    A->n = n;
    A->nnz = (int64_t)ci.size();
    std::vector<int> offs;
    std::vector<double> dv;
    std::vector<double> dcv;
    build_dia(n, rp, ci, v, offs, dv, A->dld, dcv, A->toep);
    hipError_t e = hipSetDevice(c->device);
    if (e == hipSuccess) e = hipMalloc(&A->rowptr, (n + 1) * sizeof(int));
    if (e == hipSuccess) e = hipMalloc(&A->col, std::max<int64_t>(A->nnz, 1) * sizeof(int));
    if (e == hipSuccess) e = hipMalloc(&A->val, std::max<int64_t>(A->nnz, 1) * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(A->rowptr, rp.data(), (n + 1) * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess && A->nnz) e = hipMemcpy(A->col, ci.data(), A->nnz * sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess && A->nnz) e = hipMemcpy(A->val, v.data(), A->nnz * sizeof(double), hipMemcpyHostToDevice);
    if (e == hipSuccess && !offs.empty()) {
        A->ndiag = (int)offs.size();
        A->hl = std::max(0, -offs.front());
        A->hu = std::max(0, offs.back());
        offs.resize(dia_rows(A->ndiag), 0);
        e = hipMalloc(&A->doff, offs.size() * sizeof(int));
        if (e == hipSuccess) e = hipMalloc(&A->dval, dv.size() * sizeof(double));
        if (e == hipSuccess) e = hipMemcpy(A->doff, offs.data(), offs.size() * sizeof(int), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMemcpy(A->dval, dv.data(), dv.size() * sizeof(double), hipMemcpyHostToDevice);
        if (e == hipSuccess) e = hipMalloc(&A->dconst, dcv.size() * sizeof(double));
        if (e == hipSuccess) e = hipMemcpy(A->dconst, dcv.data(), dcv.size() * sizeof(double), hipMemcpyHostToDevice);
    }
    if (e == hipSuccess && offs.empty()) {
        std::vector<long long> sptr;
        std::vector<int> sw, rl, sc;
        std::vector<double> sv;
        if (build_sell(n, rp, ci, v, sptr, sw, rl, sc, sv)) {
            A->sell = 1;
            e = hipMalloc(&A->sptr, sptr.size() * sizeof(long long));
            if (e == hipSuccess) e = hipMalloc(&A->swidth, sw.size() * sizeof(int));
            if (e == hipSuccess) e = hipMalloc(&A->rowlen, rl.size() * sizeof(int));
            if (e == hipSuccess) e = hipMalloc(&A->scol, std::max<size_t>(sc.size(), 1) * sizeof(int));
            if (e == hipSuccess) e = hipMalloc(&A->sval, std::max<size_t>(sv.size(), 1) * sizeof(double));
            if (e == hipSuccess) e = hipMemcpy(A->sptr, sptr.data(), sptr.size() * sizeof(long long), hipMemcpyHostToDevice);
            if (e == hipSuccess) e = hipMemcpy(A->swidth, sw.data(), sw.size() * sizeof(int), hipMemcpyHostToDevice);
            if (e == hipSuccess) e = hipMemcpy(A->rowlen, rl.data(), rl.size() * sizeof(int), hipMemcpyHostToDevice);
            if (e == hipSuccess && !sc.empty()) e = hipMemcpy(A->scol, sc.data(), sc.size() * sizeof(int), hipMemcpyHostToDevice);
            if (e == hipSuccess && !sv.empty()) e = hipMemcpy(A->sval, sv.data(), sv.size() * sizeof(double), hipMemcpyHostToDevice);
        }
    }
    if (e != hipSuccess) {
        free_mat(A);
        return fail(TK_ERR_ALLOC, "matrix upload: %s", hipGetErrorString(e));
    }
    c->refs++;
    *out = A;
    return TK_OK;
}

tk_status tk_matrix_from_csc(tk_ctx* c, int64_t n, const int64_t* colptr, const int64_t* rowval,
                             const double* nzval, int one_based, tk_mat** out) { TK_API_BEGIN
    CHECKARG(c && colptr && out && n > 0, "bad argument");
    const int64_t base = one_based ? 1 : 0;
    const int64_t nnz = colptr[n] - colptr[0];
    CHECKARG(nnz >= 0 && nnz < (int64_t)INT32_MAX, "nnz out of range");
    CHECKARG(nnz == 0 || (rowval && nzval), "rowval/nzval NULL");
    // CSC -> CSR: scanning columns in ascending order leaves every row's entries in
    // ascending column order, i.e. the order Julia's scatter mul! adds them.
    std::vector<int> rp(n + 1, 0), ci(nnz);
    std::vector<double> v(nnz);
    for (int64_t p = 0; p < nnz; ++p) {
        const int64_t r = rowval[p] - base;
        if (r < 0 || r >= n) return fail(TK_ERR_ARG, "row index %lld out of range", (long long)rowval[p]);
        rp[r + 1]++;
    }
    for (int64_t i = 0; i < n; ++i) rp[i + 1] += rp[i];
    std::vector<int> fill(rp.begin(), rp.end() - 1);
    for (int64_t j = 0; j < n; ++j) {
        const int64_t p0 = colptr[j] - colptr[0], p1 = colptr[j + 1] - colptr[0];
        if (p1 < p0) return fail(TK_ERR_ARG, "colptr not monotone at %lld", (long long)j);
        for (int64_t p = p0; p < p1; ++p) {
            const int64_t r = rowval[p] - base;
            const int q = fill[r]++;
            ci[q] = (int)j;
            v[q] = nzval[p];
        }
    }
    return upload_csr(c, n, rp, ci, v, out);
    TK_API_END
}

tk_status tk_matrix_from_csr(tk_ctx* c, int64_t n, const int64_t* rowptr, const int64_t* colind,
                             const double* val, int one_based, tk_mat** out) { TK_API_BEGIN
    CHECKARG(c && rowptr && out && n > 0, "bad argument");
    const int64_t base = one_based ? 1 : 0;
    const int64_t nnz = rowptr[n] - rowptr[0];
    CHECKARG(nnz >= 0 && nnz < (int64_t)INT32_MAX, "nnz out of range");
    std::vector<int> rp(n + 1), ci(nnz);
    std::vector<double> v(nnz);
    for (int64_t i = 0; i <= n; ++i) rp[i] = (int)(rowptr[i] - rowptr[0]);
    for (int64_t i = 0; i < n; ++i) {
        int64_t last = -1;
        for (int64_t p = rp[i]; p < rp[i + 1]; ++p) {
            const int64_t cc = colind[p] - base;
            if (cc < 0 || cc >= n) return fail(TK_ERR_ARG, "column index out of range in row %lld", (long long)i);
            if (cc <= last) return fail(TK_ERR_ARG, "row %lld: columns not strictly ascending", (long long)i);
            last = cc;
            ci[p] = (int)cc;
            v[p] = val[p];
        }
    }
    return upload_csr(c, n, rp, ci, v, out);
    TK_API_END
}

static void mat_release(tk_mat* A) {
    if (--A->refs > 0) return;
    tk_ctx* c = A->ctx;
    hipSetDevice(c->device);
    if (!c->stuck) sync_bounded(c, c->stream, "tk_matrix_destroy");
    if (!c->stuck) free_mat(A);   // (stuck: device buffers left to process exit)
    ctx_release(c);
}

tk_status tk_matrix_destroy(tk_mat* A) { TK_API_BEGIN
    if (!A) return TK_OK;
    mat_release(A);
    return TK_OK;
    TK_API_END
}

int tk_matrix_format(tk_mat* A) { return A ? (A->ndiag > 0 ? A->ndiag : (A->sell ? -2 : 0)) : -1; }

tk_status tk_matvec(tk_mat* A, const double* x, double* y) { TK_API_BEGIN
    CHECKARG(A && x && y, "NULL argument");
    tk_ctx* c = A->ctx;
    HIPCHK(hipSetDevice(c->device));
    double *dx = nullptr, *dy = nullptr;
    HIPCHK(hipMalloc(&dx, A->n * sizeof(double)));
    hipError_t e = hipMalloc(&dy, A->n * sizeof(double));
    if (e == hipSuccess) e = hipMemcpyAsync(dx, x, A->n * sizeof(double), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) {
        launch_spmv(A->spm(), dx, dy, c->stream);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(y, dy, A->n * sizeof(double), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    hipFree(dx);
    hipFree(dy);
    if (e != hipSuccess) return fail(TK_ERR_HIP, "tk_matvec: %s", hipGetErrorString(e));
    return TK_OK;
    TK_API_END
}

// ------------------------------------------------------------------ decomposition
struct tk_decomp {
    tk_ctx* ctx;
    int method, d_total, foff, nf, kmax, m, nvmax;
    int64_t n, ld;
    int ntiles, npart;
    int jnext = 0;          // next step index
    int fmt = 0;            // SpMV storage shared by all local factors (KArgs::fmt)
    bool onesweep = false;  // Arnoldi as one sweep per step (k_arn_d1): banded A_s only
    bool fin_d = true;      // ungated column writes through k_fin_d (TKHIP_FIN_D=0: tile-loop kernels)
    int npd = 0;            // max DFac::npd over the local factors (grid width of k_arn_d1)
    int nwl = 0;            // max DFac::nwl (grid width of k_lan_1w)
    bool inited = false;
    bool pending = false;   // last step's column j+1 not yet written (fused pipeline)
    bool in_sweep = false;  // inside tk_decomp_sweep: one timing pair for the whole sweep
    bool failed = false;    // a step returned an error: later steps are refused
    int fail_step = -1;     // TKHIP_TEST_FAIL_STEP=j at create: step j reports an error (tests)
    int skip_mask = 0;      // TKHIP_TEST_SKIP (timing experiments only, wrong results): 1 reduce, 2 post
    // one-sweep Arnoldi: the bookkeeping of step bk_j (its record, H column, signals) has not
    // been enqueued yet; the next step's k_arn_d1 runs it in a spare block (bk_args = the
    // step's KArgs), or bk_flush launches it on its own
    int bk_j = -1;
    int bk_kind = 0;        // 0: k_arn_d1's bookkeeping (POST_ARN_D), 1: k_lan_1w's record signal
    KArgs bk_args;
    bool mfspmv = false;    // CGS2 factors sharing one A_s: one gather per nonzero for all (k_spmv_mf)
    // orthogonality_data of global factor 0 (src/tensor_krylov_method.jl:103) from one MFMA SYRK
    // of its basis when asked (tk_decomp_gram) instead of a Gram row per step (TKHIP_GRAM)
    bool gram_deferred = false;
    bool any_gram = false;   // some local factor keeps a per-step Gram row
    // single-column basis tiles (KArgs::sl): the Gram-free one-sweep TensorLanczos, whose step
    // reads one column and writes one (TKHIP_LANCZOS_SL=0 keeps the paired columns)
    bool sl = false;
    double* gram_scr = nullptr;
    bool gram_scr_owned_by_allocs = false;   // (allocated at create: freed with allocs)
    // the Gram values land in host-mapped memory, then a sequence word (k_mirror_records, as
    // the records): the host spins on the word instead of a copy + stream sync (that path
    // cost ~7-9 ms at its first use in a process, inside the driver loop)
    double* gram_host = nullptr;
    unsigned long long* gram_done = nullptr;
    unsigned long long gram_seq = 0;
    // the SYRK runs on a stream of its own (it only reads finished columns), so it overlaps
    // what the caller enqueues next -- the flush + V*Y of the solve's end; a new sequence
    // (tk_decomp_init) waits for it before rewriting the basis
    hipEvent_t gev_in = nullptr, gev_done = nullptr;   // (the context's Gram stream)
    // Factor groups (one-sweep Arnoldi / Gram-free Lanczos, nf >= 2): the local factors step as
    // 2 (default) or 3 groups, each on its own stream (grp_stream), each in its own launches,
    // so one group's launch drain and reduce overlap the other's sweep (two C2 halves on two
    // streams: 7 % less time than one 8-factor launch per step, tools/stream_probe.py).  The
    // streams fork at the first grouped step and join before anything else touches the
    // decomposition (fork_groups / join_groups).
    // ngr groups (1: none; TKHIP_FACTOR_GROUPS=3: three): group g steps local factors
    // [gst[g], gst[g+1]) on grp_stream(g) -- the compute stream, fstream, gstream
    int ngr = 1;
    int gst[4] = {0, 0, 0, 0};
    bool forked = false;
    hipEvent_t fev_fork = nullptr, fev_join[2] = {nullptr, nullptr};
    bool gram_inflight = false;
    // the Gram launched ahead by tk_decomp_gram_ahead (0: none for this sequence): its column
    // count and the sequence number its host mirror publishes
    int ahead_k = 0;
    unsigned long long ahead_want = 0;
    double* Uint = nullptr;
    bool bk_fold = true;    // TKHIP_BK_FOLD=0: every step's bookkeeping as its own k_post
    // fused one-sweep Arnoldi launches (TKHIP_D1_FUSE): step j's reduce runs in the leading blocks
    // of step j+1's launch instead of a launch of its own; red_j = the step whose partials are not
    // reduced yet (-1 none; red_flush launches k_reduce256 for it), wseq = the last step word
    bool fuse = false;
    int red_j = -1;
    unsigned long long wseq = 0;
    unsigned int* werr = nullptr;           // host-mapped: a fused wait gave up (never, if healthy)
    // exchange signalling without compute-queue markers: k_post blocks add to *xflag, the
    // exchange stream waits (hipStreamWaitValue64) for xcount
    unsigned long long* xflag = nullptr;
    unsigned long long xcount = 0;
    // records exchange: one signal word per local factor (DFac::xsig, zeroed at create), set
    // by each step's k_post / bookkeeping block to the step's xval; a slot is complete when every
    // factor's word shows xscnt[slot]
    std::vector<unsigned long long*> xsig;
    std::vector<unsigned long long> xscnt;   // per slot: the xval of the step that writes it
    unsigned long long xsq = 0, cur_xval = 0;
    // TKHIP_TEST_GROUP_DELAY_US (tests, read at create): group 0's stream held back this long
    // before each grouped launch, so the other groups run steps ahead of it
    double gdelay_us = 0.0;
    // single rank: records also land in host-mapped memory with a per-factor sequence word,
    // so tk_decomp_records waits for exactly its steps (not for the whole queue)
    double* hrec = nullptr;                 // [(kmax+2) slots][d_total][m]
    unsigned long long* hdone = nullptr;    // [(kmax+2) slots][nf]
    unsigned long long seq = 0;
    std::vector<unsigned long long> slot_seq;   // per slot: seq of the signalled step that wrote it, 0 = none
    // multi-rank: each exchanged slot is mirrored to hrec by the exchange stream, xdone[slot]
    // = its sequence number (host-mapped); xslot_seq[slot] = the number to wait for
    unsigned long long* xdone = nullptr;
    std::vector<unsigned long long> xslot_seq;
    // which slots go through which all-reduce (tk_xsched.h): the slots of xs.group
    // consecutive steps (TKHIP_XCH_GROUP, default 4, agreed over the ranks at create) per
    // call; xev[slot] = the slot whose ev_x marks the exchange that carried it; xcnt[slot] =
    // the signal count (xcount) at which the slot's record is written
    XSched xs;
    std::vector<int> xev;
    std::vector<unsigned long long> xcnt;
    // TKHIP_TEST_XCH_STALL=s (tests): the exchange of the range holding slot s waits on a
    // word nobody writes until a reader's deadline expires (a peer that never joins)
    int stall_slot = -1;
    unsigned long long* stallw = nullptr;
    unsigned long long stall_v = 0;
    hipStream_t cstream = nullptr;          // record copies (multi-rank): no wait on the compute queue
    int last_j = -1;
    std::vector<tk_mat*> mats;
    std::vector<DFac> hf;   // host copy of descriptors
    DFac* df = nullptr;     // device descriptors
    std::vector<void*> allocs;
    double* rec = nullptr;   // send records [(kmax+2) slots][d_total][m] (local rows only)
    double* recv = nullptr;  // all-reduced records (== rec on a single rank)
    // multi-rank: the send rows alternate between two buffers by sequence (tk_decomp_init
    // swaps rec / rec_alt and the slot-guard state with them), so a sequence's steps never
    // wait for the previous sequence's all-reduces to finish reading their rows -- only the
    // ones of two sequences back, long done unless the host runs a whole sequence ahead
    double* rec_alt = nullptr;
    std::vector<unsigned long long> xslot_seq_alt;
    std::vector<int> xev_alt;
    // replica of factors another rank owns (exp-sum-term split, tk_decomp_set_replica): the
    // all-reduce sends these zero rows instead of rec, so every record is counted once
    double* zrec = nullptr;
    double* Ydev = nullptr; size_t ycap = 0;
    double* Xdev = nullptr; size_t xcap = 0;
    double* scratch = nullptr;   // column gather buffer (n x 8)
    // per-slot events: compute -> exchange (slot written) and exchange -> compute
    // (the all-reduce has finished reading the slot's send rows)
    std::vector<hipEvent_t> ev_c, ev_x;
    // slot guards: how often each ev_x was recorded, and the (event, record) the compute stream
    // last waited for -- the slots of one exchange share its event, so one wait packet covers
    // them all (a barrier packet per step cost the host-ahead bench sweeps ~2-3 us per step)
    std::vector<unsigned> ev_x_gen;
    int guard_ev = -1;
    unsigned guard_gen = 0;
};

int tk_record_len(int kmax) { return rec_len(kmax); }

static tk_status dalloc(tk_decomp* dc, void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
    if (e != hipSuccess) return fail(TK_ERR_ALLOC, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
    dc->allocs.push_back(*p);
    e = hipMemset(*p, 0, std::max<size_t>(bytes, 16));
    if (e != hipSuccess) return fail(TK_ERR_HIP, "hipMemset: %s", hipGetErrorString(e));
    return TK_OK;
}

static void free_decomp(tk_decomp* dc) {
    if (dc->ctx->stuck) {   // a collective may still read or write these buffers
        delete dc;
        return;
    }
    for (hipEvent_t e : dc->ev_c) hipEventDestroy(e);
    for (hipEvent_t e : dc->ev_x) hipEventDestroy(e);
    for (void* p : dc->allocs) hipFree(p);
    if (dc->scratch) hipFree(dc->scratch);
    if (dc->Ydev) hipFree(dc->Ydev);
    if (dc->Xdev) hipFree(dc->Xdev);
    if (dc->gram_scr && !dc->gram_scr_owned_by_allocs) hipFree(dc->gram_scr);
    if (dc->gram_host) hipHostFree(dc->gram_host);
    if (dc->gram_done) hipHostFree(dc->gram_done);
    if (dc->xflag) hipFree(dc->xflag);
    for (unsigned long long* p : dc->xsig) hipFree(p);
    if (dc->stallw) hipFree(dc->stallw);
    if (dc->hrec) hipHostFree(dc->hrec);
    if (dc->hdone) hipHostFree(dc->hdone);
    if (dc->xdone) hipHostFree(dc->xdone);
    if (dc->cstream) hipStreamDestroy(dc->cstream);
    if (dc->fev_fork) hipEventDestroy(dc->fev_fork);
    for (hipEvent_t e : dc->fev_join)
        if (e) hipEventDestroy(e);
    if (dc->gev_in) hipEventDestroy(dc->gev_in);
    if (dc->gev_done) hipEventDestroy(dc->gev_done);
    delete dc;
}

// ------------------------------------------------------------------ reduce hand-off self-check
// (Since round 5 the separate one-sweep Arnoldi reduce is a plain reduction: its readers
// evaluate the scalars themselves.  What still hands values between the blocks of one launch is
// the fused launch -- the reducers' values to the windows through the step word -- and the
// one-sweep Lanczos reduce's last block; the check's job runs fused.)
// k_reduce256 hands a one-sweep step's reduced values to the block that evaluates the next
// step's scalars through agent-scope relaxed atomics -- correct on gfx950 by measurement
// (/opt/skills/guides/MI355X_MICROARCH.md's hand-off table), not by the HIP memory model,
// whose own form (release/acquire add, acquire fence: an L2 writeback and invalidate per
// value block) costs C2 5 %, C1 12 % (profiles/r04/reduce_handoff_mm_ab.txt).  Before the first
// decomposition of a process whose steps use it, both forms run the same small one-sweep
// Arnoldi job (two factors, n = 2^18: 1 041 window blocks publishing partials, 24 steps, on a
// context of its own: no collective, nothing queued on the caller's streams) and must give
// bitwise the same records; on any difference -- or if the check cannot run -- the process
// keeps the memory-model form.  TKHIP_RED_MM=0/1 skips the check and forces
// a form.  tk_reduce_handoff() reports the outcome.
// 0 not checked, 1 relaxed (checked), 2 MM (the forms differed), 3 forced (TKHIP_RED_MM), 4 MM (the
// check could not run: context, matrix or decomposition creation, or a step, failed)
static std::atomic<int> g_red_state{0};
static std::atomic<double> g_red_check_ms{0.0};   // the check's wall time (setup cost of the first create)
static thread_local bool g_in_red_check = false;

static int red_check_run(int device) {
    const int64_t n = 1 << 18;
    const int K = 24, nf = 2;
    std::vector<int64_t> colptr(n + 1), rowval;
    std::vector<double> nz;
    rowval.reserve(3 * n);
    nz.reserve(3 * n);
    for (int64_t j = 0; j < n; ++j) {   // tridiagonal (-1, 2, -1), column by column
        colptr[j] = (int64_t)rowval.size();
        for (int64_t i = j - 1; i <= j + 1; ++i)
            if (i >= 0 && i < n) {
                rowval.push_back(i);
                nz.push_back(i == j ? 2.0 : -1.0);
            }
    }
    colptr[n] = (int64_t)rowval.size();
    std::vector<double> b0(n), b1(n);
    for (int64_t i = 0; i < n; ++i) {
        b0[i] = 1.0 + 0.5 * sin(0.001 * (double)i);
        b1[i] = 1.0 + 0.25 * cos(0.003 * (double)i) + 1e-3 * (double)(i % 7);
    }
    tk_ctx* cc = nullptr;
    tk_mat* A = nullptr;
    tk_decomp* dc = nullptr;
    int verdict = 4;   // (could not run, unless both forms ran)
    std::vector<double> rec[2];
    if (tk_ctx_create(device, &cc) == TK_OK &&
        tk_matrix_from_csc(cc, n, colptr.data(), rowval.data(), nz.data(), 0, &A) == TK_OK) {
        tk_mat* mats[2] = {A, A};
        const double* bs[2] = {b0.data(), b1.data()};
        if (tk_decomp_create(cc, TK_ARNOLDI, nf, 0, nf, mats, bs, n, K, 0, &dc) == TK_OK &&
            tk_decomp_arnoldi_sweeps(dc) == 1) {
            bool ok = true;
            for (int mode = 0; mode < 2 && ok; ++mode) {
                set_red_mm(mode);
                rec[mode].assign((size_t)(K + 1) * nf * rec_len(K), 0.0);
                ok = tk_decomp_init(dc, nullptr) == TK_OK && tk_decomp_sweep(dc, 0, K) == TK_OK &&
                     tk_decomp_records(dc, 0, K + 1, rec[mode].data()) == TK_OK;
            }
            if (ok) verdict = memcmp(rec[0].data(), rec[1].data(), rec[0].size() * sizeof(double)) == 0 ? 1 : 2;
        }
    }
    if (dc) tk_decomp_destroy(dc);
    if (A) tk_matrix_destroy(A);
    if (cc) tk_ctx_destroy(cc);
    return verdict;
}

static void red_check_once(int device) {
    if (g_in_red_check) return;
    int exp = 0;
    if (!g_red_state.compare_exchange_strong(exp, -1)) {
        while (g_red_state.load() < 0) std::this_thread::yield();   // (another thread is checking)
        return;
    }
    if (const char* e = getenv("TKHIP_RED_MM")) {
        set_red_mm(e[0] == '1');
        g_red_state.store(3);
        return;
    }
    g_in_red_check = true;
    const auto t0 = std::chrono::steady_clock::now();
    const int v = red_check_run(device);
    g_red_check_ms.store(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    g_in_red_check = false;
    set_red_mm(v == 1 ? 0 : 1);
    if (v != 1)
        fprintf(stderr, "libtkhip: the relaxed reduce hand-off %s: using the memory-model form\n",
                v == 2 ? "gave other records than the memory-model form in its self-check"
                       : "self-check could not run");
    g_red_state.store(v);
}

// 0: the relaxed hand-off, self-checked; 1: the memory-model form (the check found a difference, or
// TKHIP_RED_MM=1); 2: relaxed, forced by TKHIP_RED_MM=0 (no check); 3: the memory-model form because
// the check could not run; -1: not settled yet
int tk_reduce_handoff(void) {
    const int st = g_red_state.load();
    if (st <= 0) return -1;
    if (st == 4) return 3;
    return red_mm() ? 1 : (st == 3 ? 2 : 0);
}

double tk_reduce_check_ms(void) { return g_red_check_ms.load(); }

tk_status tk_decomp_create(tk_ctx* c, int method, int d_total, int first_factor, int nf,
                           tk_mat* const* mats, const double* const* b, int64_t n, int kmax,
                           int track_all_gram, tk_decomp** out) { TK_API_BEGIN
    CHECKARG(c && out && (nf == 0 || (mats && b)), "NULL argument");
    // (the one-sweep steps' reduce hand-off form, settled once per process)
    if (method != TK_LANCZOS_REORTH) red_check_once(c->device);
    CHECKARG(method >= TK_ARNOLDI && method <= TK_LANCZOS_REORTH, "unknown method");
    // nf == 0: a rank of a job with more ranks than factors (it only takes part in the
    // records all-reduce; every launch is skipped)
    CHECKARG(nf >= 0 && d_total >= 1 && first_factor >= 0 && first_factor + nf <= d_total, "bad factor range");
    CHECKARG(kmax >= 1 && kmax <= 1000, "kmax out of range [1, 1000]");
    CHECKARG(n >= 1, "n must be positive");
    for (int f = 0; f < nf; ++f) {
        CHECKARG(mats[f] && b[f], "NULL matrix or rhs");
        if (mats[f]->n != n) return fail(TK_ERR_ARG, "factor %d has order %lld != n = %lld", f, (long long)mats[f]->n, (long long)n);
        if (mats[f]->ctx != c) return fail(TK_ERR_ARG, "factor %d matrix belongs to another context", f);
    }
    HIPCHK(hipSetDevice(c->device));
    tk_decomp* dc = new tk_decomp();
    dc->ctx = c;
    dc->method = method;
    dc->d_total = d_total;
    dc->foff = first_factor;
    dc->nf = nf;
    dc->kmax = kmax;
    dc->m = rec_len(kmax);
    dc->n = n;
    dc->ld = (n + 255) / 256 * 256;
    dc->ntiles = (int)((n + 255) / 256);
    // partial count: a function of n only (bitwise results independent of the factor
    // partition); TKHIP_NPART overrides it for tuning experiments
    int npcap = 1024;
    {
        const char* e = getenv("TKHIP_NPART");
        npcap = e ? std::max(32, atoi(e)) : 1024;
        dc->npart = std::min(dc->ntiles, npcap);
    }
    {
        auto fmt_of = [](const tk_mat* A) { return A->ndiag > 0 ? (A->ndiag <= 4 ? (A->toep ? 5 : 1) : 4) : (A->sell ? 2 : 3); };
        dc->fmt = nf > 0 ? fmt_of(mats[0]) : 0;
        for (int f = 1; f < nf; ++f)
            if (fmt_of(mats[f]) != dc->fmt) dc->fmt = 0;
    }
    // Arnoldi runs as one sweep per step (k_arn_d1) when every local factor is banded
    // (DIA, bandwidths <= 4: the SpMVs read their vector from the window in LDS) and its
    // basis is addressable with 31-bit offsets; TKHIP_ARNOLDI=cgs2 keeps the two-sweep CGS2.
    // TensorLanczos likewise (k_lan_1s: TTR with the orthogonalization against v_j delayed a
    // step); TKHIP_LANCZOS=ttr keeps the three-pass TTR kernels.
    {
        const char* e = getenv("TKHIP_ARNOLDI");
        const char* el = getenv("TKHIP_LANCZOS");
        bool ok = ((method == TK_ARNOLDI && !(e && strcmp(e, "cgs2") == 0)) ||
                   (method == TK_LANCZOS && !(el && strcmp(el, "ttr") == 0))) &&
                  (dc->fmt == 1 || dc->fmt == 5);
        const double vbytes = (double)dc->ntiles * 256 * ((kmax + 2) & ~1) * sizeof(double);
        ok = ok && vbytes < 2147483648.0 - 1048576.0;
        for (int f = 0; ok && f < nf; ++f) ok = mats[f]->hl <= 4 && mats[f]->hu <= 4;
        dc->onesweep = ok;
    }
    dc->nvmax = dc->onesweep ? 3 * kmax + 8 : 2 * kmax + 8;
    {
        // fused one-sweep Arnoldi launches: TKHIP_D1_FUSE=1 on, 0 off; results are bitwise those
        // of the separate reduce launch (the same reduction, the same coefficients).  Unset: on
        // when the local factors step as factor groups (two streams) over at most
        // TKHIP_D1_FUSE_WINDOWS (2048) windows in all -- C4 at N = 8 / 4 (2 / 3 factors of 525
        // windows: +6..16 % / +3 %); off for one factor (C4 rank 7 -1..3 %, C2 N = 8 -7 %) and for
        // larger grids (C4 N = 1's 5250 windows -9 %, C2 N = 2 / 4 -8..11 %), where the window
        // blocks waiting for the reducers cost more than the launch they save
        // (profiles/r05/fused_launch_ab*.txt)
        const char* e = getenv("TKHIP_D1_FUSE");
        bool want = e ? e[0] == '1' : false;
        if (!e) {
            const char* eg = getenv("TKHIP_FACTOR_GROUPS");
            const char* ew = getenv("TKHIP_D1_FUSE_WINDOWS");
            const long wmax = ew ? atol(ew) : 2048;
            long wins = 0;
            for (int f = 0; f < nf; ++f) {
                const int ws = 256 - 2 * (mats[f]->hl + mats[f]->hu);
                wins += ws > 0 ? (long)((n + ws - 1) / ws) : 0;
            }
            want = nf >= 2 && !(eg && atoi(eg) <= 1) && wins <= wmax;
        }
        // (the hand-off self-check's own job: the fused launches are what hand values between
        // the blocks of one launch -- the separate reduce is a plain reduction since round 5)
        if (g_in_red_check) want = true;
        dc->fuse = method == TK_ARNOLDI && dc->onesweep && nf > 0 && want;
    }
    {
        const char* e = getenv("TKHIP_FIN_D");
        dc->fin_d = !(e && e[0] == '0');
    }
    {
        // Gram rows per step (the loss check of LanczosReorth needs them; track_all_gram asks
        // for every factor's) or one SYRK of factor 0's basis at the end (k <= 64 columns on
        // MFMA), the default: the one-sweep Lanczos step reads no basis row, so a per-step Gram
        // row streams the tracked factor's whole basis every step; for Arnoldi the row's dots
        // make the tracked factor's launch the long pole at one factor per GPU (TKHIP_GRAM=rows
        // restores the rows)
        const char* e = getenv("TKHIP_GRAM");
        bool def = true;
        if (e && strcmp(e, "rows") == 0) def = false;
        if (e && strcmp(e, "deferred") == 0) def = true;
        if (track_all_gram == 2) def = false;   // the caller reads factor 1's loss every step
        dc->gram_deferred = def && method != TK_LANCZOS_REORTH && !track_all_gram && kmax + 1 <= 64;
    }
    dc->mats.assign(mats, mats + nf);
    dc->hf.resize(nf);
    const int KP = kmax + 2, KC = kmax + 1;
    tk_status st = TK_OK;
    {
        // CGS2 over factors that share one gather-format A_s (TKHIP_MFSPMV=0 turns it off)
        const char* e = getenv("TKHIP_MFSPMV");
        bool ok = method == TK_ARNOLDI && !dc->onesweep && nf >= 2 && nf <= 8 && (dc->fmt == 2 || dc->fmt == 3) &&
                  !(e && e[0] == '0');
        for (int f = 1; ok && f < nf; ++f) ok = mats[f] == mats[0];
        dc->mfspmv = ok;
    }
#define DA(ptr, bytes)                                          \
    do {                                                        \
        void* p_ = nullptr;                                     \
        st = dalloc(dc, &p_, (bytes));                          \
        if (st != TK_OK) { free_decomp(dc); return st; }        \
        ptr = (decltype(ptr))p_;                                \
    } while (0)
    for (int f = 0; f < nf; ++f) {
        DFac& d = dc->hf[f];
        d.A = mats[f]->spm();
        d.hl = mats[f]->hl;
        d.hu = mats[f]->hu;
        {
            // overlapping windows of 256 rows owning 256 - 2(hl+hu), one k_arn_d1 block (and
            // one partial slot) each: a function of (n, hl, hu) only
            const int ws = 256 - 2 * (d.hl + d.hu);
            d.nwin = (int)((n + ws - 1) / ws);
            d.npd = d.nwin;
        }
        dc->npd = std::max(dc->npd, d.npd);
        d.nwl = lan_windows(n, d.hl, d.hu);
        dc->nwl = std::max(dc->nwl, d.nwl);
        // partial slots: CGS2 (npart), one-sweep Arnoldi windows (npd), k_lan_1w's wide windows
        // (nwl: more than ntiles when TK_LAN_RPT = 1 and the band is wide), one per tile (k_fin_d)
        const int npp = std::max(std::max(std::max(dc->npart, dc->onesweep ? d.npd : 0), dc->onesweep ? d.nwl : 0),
                                 dc->ntiles);
        DA(d.V, (size_t)dc->ntiles * 256 * ((kmax + 2) & ~1) * sizeof(double));   // tile-major, paired columns
        double* bb;
        DA(bb, (size_t)dc->ld * sizeof(double));
        hipError_t e = hipMemcpy(bb, b[f], n * sizeof(double), hipMemcpyHostToDevice);
        if (e != hipSuccess) { free_decomp(dc); return fail(TK_ERR_HIP, "upload b: %s", hipGetErrorString(e)); }
        d.b = bb;
        DA(d.W, (size_t)dc->ld * sizeof(double));
        DA(d.U, (size_t)dc->ld * sizeof(double));
        // (one-sweep Arnoldi: window-major groups of D1G values, nvmax rounded up to whole groups)
        const size_t nvp = (size_t)d1_groups(dc->nvmax) * D1G;
        DA(d.P1, nvp * npp * sizeof(double));
        DA(d.P2, (size_t)dc->nvmax * npp * sizeof(double));
        DA(d.RED1, (size_t)std::max(dc->nvmax, RED1_LEN(kmax)) * sizeof(double));
        DA(d.RED2, (size_t)dc->nvmax * sizeof(double));
        DA(d.sc, SC_COUNT * sizeof(double));
        DA(d.h2, (KP + 16) * sizeof(double));   // + COEF_TAIL (tk_kernels.hip)
        DA(d.g, (KP + 16) * sizeof(double));
        DA(d.H, (size_t)KP * KC * sizeof(double));
        DA(d.lossrow, (size_t)KP * sizeof(double));
        DA(d.ctr, 16);
        d.Q = nullptr;
        d.ctrg = nullptr;
        if (dc->onesweep && method == TK_ARNOLDI) {
            DA(d.Q, (size_t)d1_groups(dc->nvmax) * 16 * D1G * sizeof(double));
            DA(d.ctrg, (size_t)d1_groups(dc->nvmax) * sizeof(unsigned int));   // (zeroed by dalloc)
        }
        DA(d.E, (size_t)(dc->onesweep ? dc->ld : 1) * sizeof(double));
        d.P1b = nullptr;
        d.rword = nullptr;
        if (dc->fuse) {
            DA(d.P1b, nvp * npp * sizeof(double));
            DA(d.rword, 64);   // (zeroed by dalloc; step words start at 1)
        }
        const int gi = first_factor + f;
        d.track_gram = (track_all_gram == 1 || method == TK_LANCZOS_REORTH || (gi == 0 && !dc->gram_deferred)) ? 1 : 0;
        dc->any_gram = dc->any_gram || d.track_gram;
        d.gidx = gi;
        d.Uint = nullptr;
        d.AU = nullptr;
        d.ifs = f;
        d.inf = nf;
        if (dc->mfspmv) {
            if (f == 0) DA(dc->Uint, (size_t)dc->ld * 8 * sizeof(double));   // rows padded (ilv_pitch <= 8)
            d.Uint = dc->Uint;
            DA(d.AU, (size_t)dc->ld * sizeof(double));
        }
    }
    {
        const char* e = getenv("TKHIP_LANCZOS_SL");
        dc->sl = method == TK_LANCZOS && dc->onesweep && dc->fin_d && !dc->any_gram && kmax <= ARN_D1_JMAX &&
                 !(e && e[0] == '0');
    }
    DA(dc->df, nf * sizeof(DFac));
    {
        hipError_t e = hipMemcpy(dc->df, dc->hf.data(), nf * sizeof(DFac), hipMemcpyHostToDevice);
        if (e != hipSuccess) { free_decomp(dc); return fail(TK_ERR_HIP, "upload descriptors: %s", hipGetErrorString(e)); }
    }
    DA(dc->rec, (size_t)(kmax + 2) * d_total * dc->m * sizeof(double));
    if (dc->fuse) dc->werr = c->werr;   // (the context's: not owned here)
    // the deferred Gram's partials (tk_decomp_gram), allocated with the rest: an allocation at
    // the first call cost up to ~15 ms inside the driver loop
    if (dc->gram_deferred && nf > 0) {
        DA(dc->gram_scr, gram_scratch_doubles(dc->ntiles) * sizeof(double));
        dc->gram_scr_owned_by_allocs = true;
        if (hipEventCreateWithFlags(&dc->gev_in, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess ||
            hipEventCreateWithFlags(&dc->gev_done, hipEventDisableTiming | hipEventDisableSystemFence) != hipSuccess) {
            free_decomp(dc);
            return fail(TK_ERR_HIP, "tk_decomp_create: gram stream / events");
        }
        void* hp = nullptr;
        void* hd = nullptr;
        if (hipHostMalloc(&hp, (size_t)gram_values(64) * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent) ==
                hipSuccess &&
            hipHostMalloc(&hd, sizeof(unsigned long long), hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
            dc->gram_host = (double*)hp;
            dc->gram_done = (unsigned long long*)hd;
            *dc->gram_done = 0;
        } else {
            if (hp) hipHostFree(hp);
            if (hd) hipHostFree(hd);
        }
        (void)hipGetLastError();
    }
    // records go through the RCCL exchange whenever factors are spread over ranks;
    // TKHIP_EXCHANGE_ALWAYS=1 takes that path on a 1-rank communicator too (tests, bench)
    if (const char* ef = TEST_ENV("TKHIP_TEST_FAIL_STEP")) dc->fail_step = atoi(ef);
    if (const char* eg = getenv("TKHIP_TEST_GROUP_DELAY_US")) dc->gdelay_us = std::max(0.0, atof(eg));
    if (const char* ek = TEST_ENV("TKHIP_TEST_SKIP")) dc->skip_mask = atoi(ek);
    if (const char* eb = getenv("TKHIP_BK_FOLD")) dc->bk_fold = eb[0] != '0';
    const char* xa = getenv("TKHIP_EXCHANGE_ALWAYS");
    if (has_peers(c) && (c->nranks > 1 || (xa && xa[0] == '1'))) {
        DA(dc->recv, (size_t)(kmax + 2) * d_total * dc->m * sizeof(double));
        DA(dc->rec_alt, (size_t)(kmax + 2) * d_total * dc->m * sizeof(double));
    } else
        dc->recv = dc->rec;
#undef DA
    if (dc->recv != dc->rec) {
        dc->ev_c.assign(kmax + 2, nullptr);
        dc->ev_x.assign(kmax + 2, nullptr);
        for (int i = 0; i < kmax + 2; ++i) {
            // ev_c (compute -> exchange, only when the signal word is unavailable) needs no
            // system-scope fence: kernel completion releases at device scope.  ev_x (exchange
            // done) keeps it: the host waits on it and then copies the received records.
            hipError_t e = hipEventCreateWithFlags(&dc->ev_c[i], hipEventDisableTiming | hipEventDisableSystemFence);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&dc->ev_x[i], hipEventDisableTiming);
            if (e != hipSuccess) {
                free_decomp(dc);
                return fail(TK_ERR_HIP, "hipEventCreate: %s", hipGetErrorString(e));
            }
        }
    }
    if (dc->recv != dc->rec && method != TK_LANCZOS_REORTH) {
        int ok = 0;
        const char* e = getenv("TKHIP_XCH_EVENTS");
        if (!(e && e[0] == '1') &&
            hipDeviceGetAttribute(&ok, hipDeviceAttributeCanUseStreamWaitValue, c->device) == hipSuccess && ok) {
            void* p = nullptr;
            if (hipExtMallocWithFlags(&p, 8, hipMallocSignalMemory) == hipSuccess && p) {
                // the count starts wherever the word is (no memset on signal memory)
                unsigned long long v0 = 0;
                if (hipMemcpy(&v0, p, 8, hipMemcpyDeviceToHost) == hipSuccess) {
                    dc->xflag = (unsigned long long*)p;
                    dc->xcount = v0;
                } else {
                    hipFree(p);
                }
            }
        }
        (void)hipGetLastError();   // an unsupported signal path must not leave a sticky error
    }
    dc->slot_seq.assign(kmax + 2, 0);
    if (dc->recv != dc->rec && dc->xflag) {
        // one signal word per local factor (signal memory is host memory): each step's k_post /
        // bookkeeping block stores the step's KArgs::xval there -- a posted store where an add was
        // a round trip the launch waited for -- and the exchange waits for every word
        // (exchange_range).  Allocation failure: the one shared word with adds
        const char* esh = TEST_ENV("TKHIP_TEST_SHARED_XSIG");
        bool okw = !(esh && esh[0] == '1');
        for (int f = 0; okw && f < nf; ++f) {
            void* p = nullptr;
            const unsigned long long zero = 0;
            okw = hipExtMallocWithFlags(&p, 8, hipMallocSignalMemory) == hipSuccess && p;
            if (okw) {
                dc->xsig.push_back((unsigned long long*)p);
                okw = hipMemcpy(p, &zero, 8, hipMemcpyHostToDevice) == hipSuccess;
            }
        }
        for (int f = 0; okw && f < nf; ++f) dc->hf[f].xsig = dc->xsig[f];
        okw = okw && hipMemcpy(dc->df, dc->hf.data(), nf * sizeof(DFac), hipMemcpyHostToDevice) == hipSuccess;
        if (!okw) {
            for (unsigned long long* p : dc->xsig) hipFree(p);
            dc->xsig.clear();
            for (int f = 0; f < nf; ++f) dc->hf[f].xsig = nullptr;
            if (hipMemcpy(dc->df, dc->hf.data(), nf * sizeof(DFac), hipMemcpyHostToDevice) != hipSuccess) {
                free_decomp(dc);
                return fail(TK_ERR_HIP, "upload descriptors");
            }
        }
        dc->xscnt.assign(kmax + 2, 0);
        (void)hipGetLastError();
    }
    {
        // with a records exchange the groups need the per-factor signal words: the exchange of
        // a step's slot then waits for every factor's word (an event marker would sit in one
        // group's stream only), and every slot guard is waited for on both group streams
        // (slot_guard)
        // One-sweep Lanczos groups its Gram-free steps (k_lan_1w + k_red_lan) the same way:
        // each launch's bookkeeping blocks mirror and signal their own group's factors (host
        // words offset by the group's first factor), k_red_lan writes only device records
        // (Lanczos groups are opt-in, TKHIP_LANCZOS_GROUPS=1: at C2 the grouped 77 us step ran
        // 8 % slower -- each group's reduce queued behind the other group's window loads;
        // profiles/r04/lanczos_groups_ab.txt)
        const char* eg = getenv("TKHIP_FACTOR_GROUPS");
        const char* elg = getenv("TKHIP_LANCZOS_GROUPS");
        const bool lan_ok = method == TK_LANCZOS && !dc->any_gram && elg && elg[0] == '1';
        const int want = eg ? std::max(1, std::min(3, atoi(eg))) : 2;
        const int G = std::min(want, nf);
        bool ok = G >= 2 && (dc->recv == dc->rec || dc->xflag) && (method == TK_ARNOLDI || lan_ok) && dc->onesweep &&
                  hipEventCreateWithFlags(&dc->fev_fork, hipEventDisableTiming | hipEventDisableSystemFence) == hipSuccess;
        for (int g = 0; ok && g < G - 1; ++g)
            ok = hipEventCreateWithFlags(&dc->fev_join[g], hipEventDisableTiming | hipEventDisableSystemFence) == hipSuccess;
        // (factor groups under an exchange need the per-factor words; TKHIP_TEST_SHARED_XSIG=1,
        // diagnostics only, runs them on the round-4 shared count)
        const char* esh = TEST_ENV("TKHIP_TEST_SHARED_XSIG");
        ok = ok && (dc->recv == dc->rec || !dc->xsig.empty() || (esh && esh[0] == '1'));
        if (ok) {
            dc->ngr = G;
            for (int g = 0; g <= G; ++g) dc->gst[g] = g * nf / G;
        }
        (void)hipGetLastError();
    }
    {
        if (dc->recv == dc->rec) {
            void* hr = nullptr;
            void* hd = nullptr;
            const size_t nrec = (size_t)(kmax + 2) * d_total * dc->m;
            if (hipHostMalloc(&hr, nrec * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
                hipHostMalloc(&hd, (size_t)(kmax + 2) * nf * sizeof(unsigned long long),
                              hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
                memset(hr, 0, nrec * sizeof(double));
                memset(hd, 0, (size_t)(kmax + 2) * nf * sizeof(unsigned long long));
                dc->hrec = (double*)hr;
                dc->hdone = (unsigned long long*)hd;
            } else {
                if (hr) hipHostFree(hr);
                if (hd) hipHostFree(hd);
            }
        } else {
            if (hipStreamCreateWithFlags(&dc->cstream, hipStreamNonBlocking) != hipSuccess) dc->cstream = nullptr;
            void* hr = nullptr;
            void* hd = nullptr;
            const size_t nrec = (size_t)(kmax + 2) * d_total * dc->m;
            if (hipHostMalloc(&hr, nrec * sizeof(double), hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
                hipHostMalloc(&hd, (size_t)(kmax + 2) * sizeof(unsigned long long),
                              hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
                memset(hr, 0, nrec * sizeof(double));
                memset(hd, 0, (size_t)(kmax + 2) * sizeof(unsigned long long));
                dc->hrec = (double*)hr;
                dc->xdone = (unsigned long long*)hd;
            } else {
                if (hr) hipHostFree(hr);
                if (hd) hipHostFree(hd);
            }
        }
        dc->xslot_seq.assign(kmax + 2, 0);
        dc->ev_x_gen.assign(kmax + 2, 0);
        dc->xcnt.assign(kmax + 2, 0);
        dc->xev.resize(kmax + 2);
        for (int i = 0; i < kmax + 2; ++i) dc->xev[i] = i;
        dc->xslot_seq_alt = dc->xslot_seq;
        dc->xev_alt = dc->xev;
        if (const char* eg = getenv("TKHIP_XCH_GROUP")) dc->xs.group = std::min(64, std::max(1, atoi(eg)));
        if (const char* es = TEST_ENV("TKHIP_TEST_XCH_STALL")) {
            void* p = nullptr;
            if (dc->recv != dc->rec && hipExtMallocWithFlags(&p, 8, hipMallocSignalMemory) == hipSuccess && p) {
                if (hipMemcpy(&dc->stall_v, p, 8, hipMemcpyDeviceToHost) == hipSuccess) {
                    dc->stallw = (unsigned long long*)p;
                    dc->stall_slot = atoi(es);
                } else {
                    hipFree(p);
                }
            }
        }
        (void)hipGetLastError();
    }
    if (dc->recv != dc->rec && c->nranks > 1) {
        // preflight: every rank must describe the same decomposition, and the exchange group
        // size is agreed (max) -- the all-reduce sequence must not depend on one rank's env
        // (the Gram mode decides whether every rank's driver joins the orthogonality
        // all-reduce at the end -- TKHIP_GRAM is read per process, so it is checked here)
        const char* names[6] = {"d_total", "kmax", "method", "n", "record length", "the Gram mode (TKHIP_GRAM)"};
        double v[7] = {(double)d_total, (double)kmax, (double)method, (double)n, (double)dc->m,
                       dc->gram_deferred ? 1.0 : 0.0, (double)dc->xs.group};
        double b[14];
        for (int i = 0; i < 7; ++i) {
            b[i] = v[i];
            b[7 + i] = -v[i];
        }
        st = host_allreduce(c, b, 14, ncclMax, "tk_decomp_create preflight");
        if (st) {
            free_decomp(dc);
            return st;
        }
        for (int i = 0; i < 6; ++i)
            if (b[i] != -b[7 + i]) {
                free_decomp(dc);
                return fail(TK_ERR_ARG, "tk_decomp_create: the %d ranks disagree on %s (min %.17g, max %.17g)",
                            c->nranks, names[i], -b[7 + i], b[i]);
            }
        dc->xs.group = (int)b[6];
    }
    c->refs++;
    for (tk_mat* A : dc->mats) A->refs++;
    *out = dc;
    return TK_OK;
    TK_API_END
}

int tk_decomp_exchange_signalled(tk_decomp* dc) { return dc && dc->xflag ? 1 : 0; }

int tk_decomp_next_step(tk_decomp* dc) { return dc ? dc->jnext : -1; }

int tk_decomp_single_columns(tk_decomp* dc) { return dc && dc->sl ? 1 : 0; }

int tk_decomp_matrix_reads(tk_decomp* dc) { return !dc ? -1 : (dc->mfspmv ? 1 : dc->nf); }

int tk_decomp_gram_deferred(tk_decomp* dc) { return dc && dc->gram_deferred ? 1 : 0; }

int tk_decomp_factor_groups(tk_decomp* dc) { return dc ? dc->ngr : 1; }

tk_status tk_decomp_set_replica(tk_decomp* dc, int replica) { TK_API_BEGIN
    CHECKARG(dc, "NULL handle");
    if (dc->inited) return fail(TK_ERR_STATE, "tk_decomp_set_replica: after tk_decomp_init");
    if (!replica) return TK_OK;
    if (dc->recv == dc->rec)
        return fail(TK_ERR_STATE, "tk_decomp_set_replica: a replica needs a records exchange (multi-rank communicator)");
    if (!dc->zrec) {
        HIPCHK(hipSetDevice(dc->ctx->device));
        void* p = nullptr;
        tk_status st = dalloc(dc, &p, (size_t)(dc->kmax + 2) * dc->d_total * dc->m * sizeof(double));
        if (st) return st;
        dc->zrec = (double*)p;
    }
    return TK_OK;
    TK_API_END
}

int tk_decomp_arnoldi_sweeps(tk_decomp* dc) {
    if (!dc) return 0;
    if (dc->method == TK_LANCZOS) return dc->onesweep ? 1 : 0;
    if (dc->method != TK_ARNOLDI) return 0;
    return dc->onesweep ? 1 : 2;
}

tk_status tk_decomp_agree(tk_decomp* dc, int* vals, int count) { TK_API_BEGIN
    CHECKARG(dc && (vals || count == 0) && count >= 0 && count <= 64, "bad argument");
    tk_ctx* c = dc->ctx;
    if (dc->recv == dc->rec || c->nranks == 1 || count == 0) return TK_OK;
    double b[64];
    for (int i = 0; i < count; ++i) b[i] = vals[i];
    tk_status st = host_allreduce(c, b, count, ncclMax, "tk_decomp_agree");
    if (st) return st;
    for (int i = 0; i < count; ++i) vals[i] = (int)b[i];
    return TK_OK;
    TK_API_END
}

tk_status tk_decomp_destroy(tk_decomp* dc) { TK_API_BEGIN
    if (!dc) return TK_OK;
    tk_ctx* c = dc->ctx;
    std::vector<tk_mat*> mats = dc->mats;
    hipSetDevice(c->device);
    // No collective starts here (a peer whose step failed never joins it): slots whose
    // group never filled are dropped -- nobody reads them.  Already enqueued exchanges are
    // waited for with the deadline.
    if (!c->stuck) sync_bounded(c, c->stream, "tk_decomp_destroy (compute stream)");
    if (!c->stuck) sync_bounded(c, c->xstream, "tk_decomp_destroy (exchange stream)");
    if (!c->stuck) sync_bounded(c, c->gstream, "tk_decomp_destroy (Gram stream)");
    if (!c->stuck) sync_bounded(c, c->fstream, "tk_decomp_destroy (factor-group stream)");
    // (the handle is released either way; a fused wait that gave up is still reported)
    const tk_status sw = dc->werr ? werr_check(c, "tk_decomp_destroy") : TK_OK;
    free_decomp(dc);
    for (tk_mat* A : mats) mat_release(A);
    ctx_release(c);
    return sw;
    TK_API_END
}

// the stream of factor group g: the compute stream, then the context's fstream and gstream
// (gstream carries the side-stream Gram only after the groups have joined)
static hipStream_t grp_stream(tk_decomp* dc, int g) {
    return g == 0 ? dc->ctx->stream : (g == 1 ? dc->ctx->fstream : dc->ctx->gstream);
}

// Before a slot's send rows are rewritten, the previous all-reduce of that slot must
// have finished reading them.
static tk_status slot_guard(tk_decomp* dc, int slot) {
    HpScope hp_(HP_GUARD);
    if (dc->recv == dc->rec) return TK_OK;
    static const bool noguard = [] {   // (TKHIP_TEST_NO_GUARD=1: timing only, records may be torn)
        const char* e = TEST_ENV("TKHIP_TEST_NO_GUARD");
        return e && e[0] == '1';
    }();
    if (noguard) return TK_OK;
    // The host-mapped mirror word answers first: an exchange is mirrored (xdone) on the
    // exchange stream right after its all-reduce, so a slot never exchanged (xslot_seq 0) or
    // whose last exchange is mirrored has no reader of its send rows left -- one host load.
    // Not mirrored yet (the host issuing ahead of the device: the bench's back-to-back sweeps,
    // the solver's steps ahead) the wait packet goes in directly; hipEventQuery cost 2-5 us of
    // host time per step there, the most of any call after the launches (TKHIP_HOST_PROFILE)
    bool need = true;
    if (dc->xdone) {
        const unsigned long long want = dc->xslot_seq[slot];
        if (want == 0 || __atomic_load_n(dc->xdone + slot, __ATOMIC_ACQUIRE) >= want) return TK_OK;
    } else {
        // (an already completed exchange needs no wait packet in the compute queue)
        HpScope hp_q(HP_GQ);
        need = hipEventQuery(dc->ev_x[dc->xev[slot]]) != hipSuccess;
    }
    const int ei = dc->xev[slot];
    if (need && ei == dc->guard_ev && dc->ev_x_gen[ei] == dc->guard_gen) need = false;   // (waited already)
    if (need) {
        dc->guard_ev = ei;
        dc->guard_gen = dc->ev_x_gen[ei];
        HIPCHK(hipStreamWaitEvent(dc->ctx->stream, dc->ev_x[dc->xev[slot]], 0));
        // factor groups already forked: the other groups' launches write their factors' rows
        // of the slot from their streams (a fork after this point inherits the wait)
        for (int g = 1; dc->forked && g < dc->ngr; ++g)
            HIPCHK(hipStreamWaitEvent(grp_stream(dc, g), dc->ev_x[dc->xev[slot]], 0));
    }
    return TK_OK;
}

// factor groups: the other groups' streams start after everything enqueued so far ...
static tk_status fork_groups(tk_decomp* dc) {
    if (dc->forked) return TK_OK;
    HIPCHK(hipEventRecord(dc->fev_fork, dc->ctx->stream));
    for (int g = 1; g < dc->ngr; ++g) HIPCHK(hipStreamWaitEvent(grp_stream(dc, g), dc->fev_fork, 0));
    dc->forked = true;
    return TK_OK;
}
// ... and the compute stream waits for them before any launch that is not a grouped step
static tk_status join_groups(tk_decomp* dc) {
    if (!dc->forked) return TK_OK;
    for (int g = 1; g < dc->ngr; ++g) {
        HIPCHK(hipEventRecord(dc->fev_join[g - 1], grp_stream(dc, g)));
        HIPCHK(hipStreamWaitEvent(dc->ctx->stream, dc->fev_join[g - 1], 0));
    }
    dc->forked = false;
    return TK_OK;
}
#define GJOIN(dc)                              \
    do {                                       \
        tk_status gj_ = join_groups(dc);       \
        if (gj_) return gj_;                   \
    } while (0)

// polls of a fused launch's bounded wait before it gives up (fuse_wait): 2^22 (~0.2 s of
// s_sleep); a test build lowers it with TKHIP_TEST_FUSE_SPIN to make the wait expire
static unsigned fuse_spin() {
#if TK_TEST_BUILD
    static const unsigned v = [] {
        const char* e = getenv("TKHIP_TEST_FUSE_SPIN");
        return e ? (unsigned)atol(e) : (1u << 22);
    }();
    return v;
#else
    return 1u << 22;
#endif
}

static KArgs base_args(tk_decomp* dc, int j, int slot) {
    KArgs a;
    a.n = dc->n;
    a.ld = dc->ld;
    a.j = j;
    a.npart = dc->npart;
    a.ntiles = dc->ntiles;
    a.kmax = dc->kmax;
    a.m = dc->m;
    a.rec = dc->rec + (size_t)slot * dc->d_total * dc->m;
    a.fmt = dc->fmt;
    a.gate = 0;
    a.ubuf = 0;
    a.xflag = nullptr;
    a.hrec = nullptr;
    a.hdone = nullptr;
    a.seq = 0;
    a.ecol = -1;
    a.mfs = 0;
    a.sl = dc->sl ? 1 : 0;
    a.red = 0;
    a.redmm = 0;
    a.wseq = 0;
    a.werr = nullptr;
    a.wspin = fuse_spin();
    a.pgrp = 0;
    a.wsc = 0;
    a.xval = 0;
    return a;
}

// One RCCL all-reduce per range of record slots: the send buffer holds only this rank's
// rows (other rows stay zero forever), so the sum is exact and every rank receives every
// factor's record.  Slots [s0, s1] are contiguous in memory, so a range is one call.
// Which ranges go out when is decided by dc->xs (tk_xsched.h), identically on every rank.
static tk_status exchange_range(tk_decomp* dc, int s0, int s1) {
    HpScope hp_(HP_XCH);
    tk_ctx* c = dc->ctx;
    STUCKCHK(c);
    const size_t cnt = (size_t)dc->d_total * dc->m;
    double* s = (dc->zrec ? dc->zrec : dc->rec) + (size_t)s0 * cnt;
    double* r = dc->recv + (size_t)s0 * cnt;
    const size_t tot = cnt * (size_t)(s1 - s0 + 1);
    // the exchange runs on its own stream, overlapping the next steps' kernels.  Step slots
    // start when the steps' k_post blocks have signalled (the count at which slot s1 was
    // written); init / flush slots and handles without the signal word after an event marker
    if (dc->xflag && s0 >= 1 && s1 <= dc->kmax) {
        if (!dc->xsig.empty()) {   // (factor groups: every factor's own count)
            for (size_t f = 0; f < dc->xsig.size(); ++f)
                HIPCHK(hipStreamWaitValue64(c->xstream, dc->xsig[f], dc->xscnt[s1],
                                            hipStreamWaitValueGte, 0xFFFFFFFFFFFFFFFFull));
        } else {
            HIPCHK(hipStreamWaitValue64(c->xstream, dc->xflag, dc->xcnt[s1], hipStreamWaitValueGte,
                                        0xFFFFFFFFFFFFFFFFull));
        }
    } else {
        HIPCHK(hipEventRecord(dc->ev_c[s1], c->stream));
        HIPCHK(hipStreamWaitEvent(c->xstream, dc->ev_c[s1], 0));
    }
    if (dc->stallw && dc->stall_slot >= s0 && dc->stall_slot <= s1)
        HIPCHK(hipStreamWaitValue64(c->xstream, dc->stallw, dc->stall_v + 1, hipStreamWaitValueGte,
                                    0xFFFFFFFFFFFFFFFFull));
    {
        // TKHIP_TEST_XCH_DELAY_US (test / prediction only): hold each all-reduce back this long
        // on the exchange stream -- what an 8-peer xGMI all-reduce costs beyond a 1-rank one --
        // so that bench.py --emulate-ranks prices collective latency
        static const double delay_us = [] {
            const char* e = getenv("TKHIP_TEST_XCH_DELAY_US");
            return e ? std::max(0.0, atof(e)) : 0.0;
        }();
        Timer tm(c, TCLS_XCH, 2, c->xstream);
        if (delay_us > 0) {
            launch_delay_us(delay_us, c->xstream);
            LAUNCHCHK("xch delay");
        }
        // TKHIP_TEST_XCH_SKIP (timing only, wrong records): 1 no mirror kernel, 2 no all-reduce
        static const int xskip = [] {
            const char* e = TEST_ENV("TKHIP_TEST_XCH_SKIP");
            return e ? atoi(e) : 0;
        }();
        HpScope hp_n(HP_NCCL);
        if (c->tcomm) {
            tk_status sx = tc_exchange(c, s, r, tot, c->xstream);
            if (sx) return sx;
        } else if (!(xskip & 2)) {
            NCCLCHK(ncclAllReduce(s, r, tot, ncclDouble, ncclSum, c->comm, c->xstream));
        }
    }
    HIPCHK(hipEventRecord(dc->ev_x[s1], c->xstream));
    ++dc->ev_x_gen[s1];
    for (int sl = s0; sl <= s1; ++sl) dc->xev[sl] = s1;
    static const bool nomirror = [] {
        const char* e = TEST_ENV("TKHIP_TEST_XCH_SKIP");
        return e && (atoi(e) & 1);
    }();
    if (dc->xdone && !nomirror) {
        ++dc->seq;
        for (int sl = s0; sl <= s1; ++sl) dc->xslot_seq[sl] = dc->seq;
        HpScope hp_m(HP_MIRROR);
        launch_mirror_records(r, dc->hrec + (size_t)s0 * cnt, (int)tot, dc->xdone + s0, s1 - s0 + 1, dc->seq,
                              c->xstream);
        LAUNCHCHK("mirror_records");
    }
    return TK_OK;
}

static tk_status xsend(tk_decomp* dc, XSched::Range r) {
    if (r.first > r.second) return TK_OK;
    for (int s = r.first; s <= r.second; ++s)
        if (!dc->xs.written(s))
            return fail(TK_ERR_STATE, "records exchange: slot %d (step %d) is not written on this rank", s, s - 1);
    return exchange_range(dc, r.first, r.second);
}

// Copy one slot's (all-reduced, on several ranks) records to the host.
static tk_status copy_slot(tk_decomp* dc, int slot, double* rec_out) {
    if (!rec_out) return TK_OK;
    GJOIN(dc);
    tk_ctx* c = dc->ctx;
    const size_t cnt = (size_t)dc->d_total * dc->m;
    if (dc->recv != dc->rec) {
        HIPCHK(hipMemcpyAsync(rec_out, dc->recv + (size_t)slot * cnt, cnt * sizeof(double), hipMemcpyDeviceToHost,
                              c->xstream));
        return sync_bounded(c, c->xstream, "records exchange", slot);
    }
    HIPCHK(hipMemcpyAsync(rec_out, dc->rec + (size_t)slot * cnt, cnt * sizeof(double), hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return TK_OK;
}

static tk_status clear_slot(tk_decomp* dc, int slot) {
    GJOIN(dc);
    double* s = dc->rec + (size_t)slot * dc->d_total * dc->m;
    HIPCHK(hipMemsetAsync(s, 0, (size_t)dc->d_total * dc->m * sizeof(double), dc->ctx->stream));
    return TK_OK;
}

#define RUN(cls, level, call, name)        \
    do {                                   \
        Timer tm_(c, cls, level);          \
        call;                              \
    } while (0);                           \
    LAUNCHCHK(name)

// TKHIP_D1_CACHE_MB: the per-step working set (MiB) up to which the one-sweep Arnoldi step
// loads the basis with the default cache policy instead of nt (0: always nt).  The Infinity
// Cache is 256 MiB; a line stays resident while everything touched between two uses fits, and
// past it the cached loads still paid up to ~450 MB (the A/B in profiles/r05/)
// TKHIP_D1_PGRP_MIN: the smallest window count per factor for window-major partials with
// factor groups (2048: C2's 4 162 windows use them, C1's 1 050 do not; 0 = always, a huge value =
// never)
static int d1_pgrp_min() {
    static const int v = [] {
        const char* e = getenv("TKHIP_D1_PGRP_MIN");
        return e ? std::max(0, atoi(e)) : 2048;
    }();
    return v;
}

static double d1_cache_bytes() {
    static const double v = [] {
        const char* e = getenv("TKHIP_D1_CACHE_MB");
        return (e ? std::max(0.0, atof(e)) : 384.0) * 1048576.0;
    }();
    return v;
}

// Step j's record is enqueued on this rank (its k_post, or the bookkeeping block of the
// next k_arn_d1): count its signal and note its host sequence number.  Local only.
static void complete_step(tk_decomp* dc, int j, unsigned long long seqj, unsigned long long xvalj) {
    if (dc->xflag) dc->xcount += (unsigned long long)dc->nf;   // one add per factor
    if (dc->hdone) dc->slot_seq[j + 1] = seqj;
    dc->xcnt[j + 1] = dc->xcount;
    if (!dc->xsig.empty()) dc->xscnt[j + 1] = xvalj;
    dc->xs.complete(j + 1);
}

// Fused one-sweep launches: the reduce of the last step, not yet run in a next launch, as a
// k_reduce256 of its own (its last block also evaluates the next step's scalars).  Local only.
static tk_status red_flush(tk_decomp* dc) {
    if (dc->red_j < 0) return TK_OK;
    if (dc->werr) {
        tk_status sw = werr_check(dc->ctx, "red_flush");
        if (sw) return sw;
    }
    GJOIN(dc);
    const int j = dc->red_j;
    dc->red_j = -1;
    tk_ctx* c = dc->ctx;
    // (a plain reduction: the fused windows and the bookkeeping evaluate the scalars)
    KArgs rx = base_args(dc, j, 0);
    rx.wsc = 1;
    if (!(dc->skip_mask & 1))
        RUN(TCLS_RED, 2, launch_reduce(dc->df, dc->nf, (j & 1) ? 5 : 1, 3 * j + 6, 0, c->stream, 0, j + 1, &rx), "reduce");
    return TK_OK;
}

// The deferred bookkeeping of the last one-sweep step as a k_post of its own.  Local only.
static tk_status bk_flush(tk_decomp* dc) {
    {
        tk_status sr = red_flush(dc);   // (its reduced values first)
        if (sr) return sr;
    }
    if (dc->bk_j < 0) return TK_OK;
    GJOIN(dc);
    tk_ctx* c = dc->ctx;
    hipStream_t s = c->stream;
    const int j = dc->bk_j;
    const KArgs ax = dc->bk_args;
    dc->bk_j = -1;
    RUN(TCLS_RED, 2, launch_post(dc->df, dc->nf, ax, dc->bk_kind ? POST_SIGNAL : POST_ARN_D, 0, 1, s), "post");
    complete_step(dc, j, ax.seq, ax.xval);
    return TK_OK;
}

// Multi-rank: slots <= S exchanged now (the deferred bookkeeping of the last step first).
static tk_status need_slots(tk_decomp* dc, int S) {
    if (dc->recv == dc->rec || S <= dc->xs.sent) return TK_OK;
    if (dc->bk_j >= 0 && dc->bk_j + 1 <= S) {
        tk_status st = bk_flush(dc);
        if (st) return st;
    }
    return xsend(dc, dc->xs.need(S));
}

tk_status tk_decomp_init(tk_decomp* dc, double* rec_out) { TK_API_BEGIN
    CHECKARG(dc, "NULL decomp");
    tk_ctx* c = dc->ctx;
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    tk_status st = dc->failed ? TK_OK : bk_flush(dc);
    if (st) return st;
    GJOIN(dc);
    dc->bk_j = -1;
    if (dc->gram_inflight) {   // (a Gram of the previous sequence still reads the basis)
        HIPCHK(hipStreamWaitEvent(s, dc->gev_done, 0));
        dc->gram_inflight = false;
    }
    static const bool rec_alt_on = [] {   // (TKHIP_REC_ALT=0: one send buffer, A/B)
        const char* e = getenv("TKHIP_REC_ALT");
        return !(e && e[0] == '0');
    }();
    if (dc->rec_alt && rec_alt_on && dc->xslot_seq.size() == dc->xslot_seq_alt.size()) {
        // (the other send buffer: its last readers are the previous-but-one sequence's)
        std::swap(dc->rec, dc->rec_alt);
        std::swap(dc->xslot_seq, dc->xslot_seq_alt);
        std::swap(dc->xev, dc->xev_alt);
    }
    st = slot_guard(dc, 0);
    if (st) return st;
    KArgs a = base_args(dc, 0, 0);
    const int nf = dc->nf;
    RUN(TCLS_PASS1, 2, launch_init_a(dc->df, nf, a, s), "init_a");
    RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, 1, dc->npart, s), "reduce");
    RUN(TCLS_RED, 2, launch_post(dc->df, nf, a, POST_INIT_A, 0, 0, s), "post");
    if (dc->onesweep) {
        RUN(TCLS_PASS1, 2, launch_init_bd(dc->df, nf, a, dc->npd, s), "init_bd");
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, 3, 0, s), "reduce");
        RUN(TCLS_RED, 2, launch_post(dc->df, nf, a, POST_INIT_B, 1, 1, s), "post");
    } else {
        RUN(TCLS_PASS1, 2, launch_init_b(dc->df, nf, a, s), "init_b");
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, 2, dc->npart, s), "reduce");
        RUN(TCLS_RED, 2, launch_post(dc->df, nf, a, POST_INIT_B, 0, 1, s), "post");
    }
    dc->inited = true;
    dc->red_j = -1;
    dc->jnext = 0;
    dc->pending = false;
    dc->last_j = -1;
    dc->ahead_k = 0;   // (a Gram launched ahead belongs to the previous sequence)
    // a new sequence: slots of the previous one that never went out are dropped (on every rank)
    dc->xs.reset();
    dc->xcnt[0] = dc->xcount;
    dc->xs.complete(0);
    if (dc->recv != dc->rec) {
        st = xsend(dc, dc->xs.need(0));
        if (st) return st;
    }
    return copy_slot(dc, 0, rec_out);
    TK_API_END
}

// write the pending column (Arnoldi / Lanczos fused pipeline)
static tk_status finalize_pending(tk_decomp* dc, const KArgs& a) {
    GJOIN(dc);
    tk_ctx* c = dc->ctx;
    hipStream_t s = c->stream;
    const int nf = dc->nf, j = a.j;
    const bool fd = dc->fin_d && j + 1 <= D1_JMAX;
    const int np = fd ? dc->ntiles : dc->npart;
    if (dc->method == TK_ARNOLDI) {
        KArgs f = a;
        if (dc->onesweep && j <= ARN_D1_JMAX) {
            f.ubuf = (j & 1) ? 0 : 1;   // one-sweep step j wrote u_{j+1} to U (j odd) or W
            f.ecol = (j & 1) ? -1 : j;  // ... and an even v_j to E
        }
        if (fd) {
            RUN(TCLS_FIN, 2, launch_fin_d(dc->df, nf, f, 0, s), "fin_d");
        } else {
            RUN(TCLS_FIN, 2, launch_arn_finalize(dc->df, nf, f, s), "arn_finalize");
        }
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 3, j + 3, np, s), "reduce");
        RUN(TCLS_RED, 2, launch_post(dc->df, nf, a, POST_ARN_FIN, 0, 1, s), "post");
    } else {
        if (fd && dc->onesweep && j <= ARN_D1_JMAX) {
            // one-sweep Lanczos: v_{j+1} = inv(beta) .* (u_j - alpha v_j) from the step's buffers
            KArgs f = a;
            f.ubuf = (j & 1) ? 0 : 1;
            f.ecol = (dc->sl || (j & 1)) ? -1 : j;   // (single columns: v_j is in V)
            RUN(TCLS_FIN, 2, launch_fin_d(dc->df, nf, f, 2, s), "fin_d");
        } else if (fd) {
            RUN(TCLS_FIN, 2, launch_fin_d(dc->df, nf, a, 1, s), "fin_d");
        } else {
            RUN(TCLS_FIN, 2, launch_lan_finalize(dc->df, nf, a, s), "lan_finalize");
        }
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, j + 3, np, s), "reduce");
        RUN(TCLS_RED, 2, launch_post(dc->df, nf, a, POST_LAN_FIN, 0, 1, s), "post");
    }
    return TK_OK;
}


static tk_status step_impl(tk_decomp* dc, int j, double* rec_out) {
    tk_ctx* c = dc->ctx;
    hipStream_t s = c->stream;
    const int nf = dc->nf, slot = j + 1;
    tk_status st = slot_guard(dc, slot);
    if (st) return st;
    KArgs a = base_args(dc, j, slot);
    KArgs ax = a;          // the step's last k_post signals the exchange stream / the host
    ax.xflag = dc->xflag;
    ax.xval = ++dc->xsq;
    dc->cur_xval = ax.xval;
    const bool hsig = dc->hdone != nullptr;
    dc->slot_seq[slot] = 0;
    if (hsig) {
        ax.hrec = dc->hrec + (size_t)slot * dc->d_total * dc->m;
        ax.hdone = dc->hdone + (size_t)slot * nf;
        ax.seq = ++dc->seq;
    }
    Timer step_timer(c, TCLS_STEP, dc->in_sweep ? 99 : 1);
    const bool grouped = dc->ngr > 1 && (dc->method == TK_ARNOLDI || (dc->method == TK_LANCZOS && !dc->any_gram)) &&
                         dc->onesweep && j <= ARN_D1_JMAX;
    if (!grouped) GJOIN(dc);
    if ((dc->method == TK_ARNOLDI || dc->method == TK_LANCZOS) && dc->onesweep && j > ARN_D1_JMAX && dc->pending &&
        dc->last_j <= ARN_D1_JMAX) {
        // leaving the one-sweep range: write the pending column v_j (its record is
        // overwritten by the CGS2 step below, which reports column j again)
        tk_status st2 = bk_flush(dc);
        if (st2) return st2;
        st2 = finalize_pending(dc, base_args(dc, j - 1, slot));
        if (st2) return st2;
        dc->pending = false;
    }
    if (dc->method == TK_ARNOLDI && dc->onesweep && j <= ARN_D1_JMAX) {
        // one sweep: writes v_j, u_{j+1}; reduce; post -> H column j and the next step's
        // coefficients.  v_j is re-derived from (U or W, h2, inv_beta) whether or not a
        // flush already wrote it (same operands, same order: the same value).
        // The step's coefficients come from the previous step's reduced dots (d1_coef); the
        // previous step's bookkeeping rides in a spare block of this launch, and this step's
        // is deferred the same way (tk_decomp_step completes the previous step's record).
        a.ubuf = j & 1;
        // one stream: the reduce is a plain reduction and the windows evaluate the scalars;
        // with factor groups the reduce's last block does (hidden behind the other group)
        a.wsc = grouped ? 0 : 1;
        // factor groups over long grids (no fused launches): window-major partials, written as
        // whole lines, and their two-level reduce (its extra hand-off hidden behind the other
        // group's sweep); short grids and one stream keep value-major partials and the one-level
        // reduce.  Both sum in the same order: bitwise the same results.  Same box, two reps
        // (profiles/r06/window_major_partials_ab.txt): C2 N = 1 +1.9 / +2.6 %, the other lines
        // within the box noise; window-major on every grouped grid (TKHIP_D1_PGRP_MIN=0): C1
        // +3.5 / -1.4 %
        a.pgrp = (grouped && !dc->fuse && dc->npd >= d1_pgrp_min()) ? 1 : 0;
        KArgs b = base_args(dc, -1, slot);
        b.j = -1;
        if (dc->bk_j >= 0 && dc->bk_j == j - 1 && dc->bk_kind == 0) b = dc->bk_args;
        else if (dc->bk_j >= 0) {
            tk_status st2 = bk_flush(dc);
            if (st2) return st2;
        }
        // the basis rows through the caches while this rank's per-step working set (every
        // local factor's V[:, 0..j) and u in / out, v_j) is at most TKHIP_D1_CACHE_MB (384): the
        // next step then re-reads much of it from the 256 MiB Infinity Cache; streamed with nt
        // beyond.  Same box, 3 repetitions (profiles/r05/vload_threshold_ab*.txt): C1 +5 %,
        // emulated C2 N = 8 +4..5 %, C4 +3 %; C2 N = 1 unchanged (its 8 factors pass 384 MB at
        // j = 3), where the default policy on every step costs 4.5 %
        const bool vcache = (double)nf * 8.0 * (double)dc->ld * (double)(j + 3) <= d1_cache_bytes();
        if (dc->fuse) {
            // step j-1's reduce in this launch's leading blocks (the pending one: nothing
            // else has read its values since); otherwise RED1 is complete already
            a.red = dc->red_j == j - 1 && j > 0 ? 1 : 0;
            if (dc->red_j >= 0 && !a.red) {
                tk_status sr = red_flush(dc);
                if (sr) return sr;
            }
            a.redmm = red_mm();
            a.wseq = a.red ? ++dc->wseq : 0;
            a.werr = dc->werr;
            dc->red_j = -1;
        }
        if (grouped) {
            // each factor group in its own launches on its own stream (the bookkeeping blocks
            // of a group's launch serve that group's factors: host-mirror words offset by g0)
            tk_status stf = fork_groups(dc);
            if (stf) return stf;
            for (int g = 0; g < dc->ngr; ++g) {
                const int g0 = dc->gst[g], ng = dc->gst[g + 1] - dc->gst[g];
                hipStream_t sg = grp_stream(dc, g);
                if (g == 0 && dc->gdelay_us > 0) {   // (tests: the other groups run ahead)
                    launch_delay_us(dc->gdelay_us, sg);
                    LAUNCHCHK("group delay");
                }
                KArgs bg = b;
                if (bg.j >= 0 && bg.hdone) bg.hdone += g0;
                {
                    Timer tm_(c, TCLS_PASS1, 2, sg);
                    HpScope hp_(HP_D1);
                    launch_arn_d1(dc->df + g0, ng, a, bg, dc->npd, dc->any_gram, vcache, dc->fuse, sg);
                }
                LAUNCHCHK("arn_d1");
                if (!(dc->skip_mask & 1) && !dc->fuse) {
                    Timer tm_(c, TCLS_RED, 2, sg);
                    HpScope hp_(HP_RED);
                    if (a.pgrp) launch_red_d1(dc->df + g0, ng, 1, j + 1, dc->npd, sg);
                    else launch_reduce(dc->df + g0, ng, 1, 3 * j + 6, 0, sg, 0, j + 1);
                }
                LAUNCHCHK("reduce");
            }
        } else {
            {
                HpScope hp_(HP_D1);
                RUN(TCLS_PASS1, 2, launch_arn_d1(dc->df, nf, a, b, dc->npd, dc->any_gram, vcache, dc->fuse, s), "arn_d1");
            }
            // (its last block per factor also evaluates the next step's scalars)
            if (!(dc->skip_mask & 1) && !dc->fuse) {
                HpScope hp_(HP_RED);
                RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, 3 * j + 6, 0, s, 0, j + 1, &a), "reduce");
            }
        }
        if (dc->fuse) dc->red_j = j;   // (reduced in the next launch, or by red_flush)
        dc->bk_j = j;
        dc->bk_args = ax;
        dc->bk_kind = 0;
        dc->pending = true;
    } else if (dc->method == TK_ARNOLDI) {
        const bool fused = dc->pending;
        if (fused) {
            if (dc->mfspmv) {
                // A U of every factor from one gather per nonzero (bitwise the per-factor SpMV)
                RUN(TCLS_PASS1, 2, launch_spmv_mf(dc->df, nf, a, s), "spmv_mf");
                a.mfs = 1;
            }
            RUN(TCLS_PASS1, 2, launch_arn_a1_fused(dc->df, nf, a, s), "arn_a1_fused");
        } else {
            if (dc->mfspmv && j == 0) {   // (k_init_b left U = v_0)
                RUN(TCLS_PASS1, 2, launch_spmv_mf(dc->df, nf, a, s), "spmv_mf");
                a.mfs = 1;
            }
            RUN(TCLS_PASS1, 2, launch_arn_a1_plain(dc->df, nf, a, s), "arn_a1_plain");
        }
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, j + 1, dc->npart, s), "reduce");
        RUN(TCLS_PASS2, 2, launch_arn_a2(dc->df, nf, a, s), "arn_a2");
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 2, 2 * j + 4, dc->npart, s), "reduce");
        RUN(TCLS_RED, 2, launch_post(dc->df, nf, ax, POST_ARN, fused ? 1 : 0, 1, s), "post");
        dc->pending = true;
    } else if (dc->method == TK_LANCZOS && dc->onesweep && j <= ARN_D1_JMAX) {
        // one sweep: writes v_j (E or its pair) and u_j; the reduce's last block takes
        // alpha_j, beta_j and writes the step's record (no post launch)
        a.ubuf = j & 1;
        if (dc->any_gram) {
            RUN(TCLS_PASS1, 2, launch_lan_1s(dc->df, nf, a, dc->npd, s), "lan_1s");
            RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, 6 + j, 0, s, 0, RED_LAN, &ax), "reduce");
        } else {
            // no Gram row: k_lan_1w's wide windows (DFac::nwl partials -- np -1 to the reduce).
            // The record's host mirror and signal are deferred to leading blocks of the next
            // step's launch (as k_arn_d1's bookkeeping): the reduce that ends the step -- on
            // the path to the next step -- then waits for no host-memory stores
            KArgs b = base_args(dc, -1, slot);
            b.j = -1;
            if (dc->bk_j >= 0 && dc->bk_j == j - 1 && dc->bk_kind == 1) b = dc->bk_args;
            else if (dc->bk_j >= 0) {
                tk_status st2 = bk_flush(dc);
                if (st2) return st2;
            }
            KArgs an = ax;
            an.xflag = nullptr;
            an.hdone = nullptr;
            an.hrec = nullptr;
            if (grouped) {
                // each factor group's window launch + reduce on its own stream (as the Arnoldi
                // groups); the leading blocks of a group's launch mirror and signal the
                // previous step's records of that group's factors: host words offset by g0
                tk_status stf = fork_groups(dc);
                if (stf) return stf;
                for (int g = 0; g < dc->ngr; ++g) {
                    const int g0 = dc->gst[g], ng = dc->gst[g + 1] - dc->gst[g];
                    hipStream_t sg = grp_stream(dc, g);
                    KArgs bg = b;
                    if (bg.j >= 0 && bg.hdone) bg.hdone += g0;
                    {
                        Timer tm_(c, TCLS_PASS1, 2, sg);
                        launch_lan_1w(dc->df + g0, ng, a, bg, dc->nwl, sg);
                    }
                    LAUNCHCHK("lan_1w");
                    {
                        Timer tm_(c, TCLS_RED, 2, sg);
                        launch_red_lan(dc->df + g0, ng, an, sg);
                    }
                    LAUNCHCHK("red_lan");
                }
            } else {
                RUN(TCLS_PASS1, 2, launch_lan_1w(dc->df, nf, a, b, dc->nwl, s), "lan_1w");
                RUN(TCLS_RED, 2, launch_red_lan(dc->df, nf, an, s), "red_lan");
            }
            dc->bk_j = j;
            dc->bk_args = ax;
            dc->bk_kind = 1;
        }
        dc->pending = true;
    } else if (dc->method == TK_LANCZOS) {
        const bool fused = dc->pending;
        if (fused && dc->fin_d && j >= 1 && j <= D1_JMAX) {
            RUN(TCLS_PASS1, 2, launch_lan_d1(dc->df, nf, a, s), "lan_d1");
            RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, j + 3, dc->ntiles, s), "reduce");
        } else if (fused) {
            RUN(TCLS_PASS1, 2, launch_lan_l1_fused(dc->df, nf, a, s), "lan_l1_fused");
            RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, j + 3, dc->npart, s), "reduce");
        } else {
            RUN(TCLS_PASS1, 2, launch_lan_l1_plain(dc->df, nf, a, s), "lan_l1_plain");
            RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, 1, dc->npart, s), "reduce");
        }
        RUN(TCLS_PASS2, 2, launch_lan_l2(dc->df, nf, a, s), "lan_l2");
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 2, 1, dc->npart, s), "reduce");
        RUN(TCLS_RED, 2, launch_post(dc->df, nf, ax, POST_LAN, fused ? 1 : 0, 1, s), "post");
        dc->pending = true;
    } else {
        // TensorLanczosReorth (src/orthogonal_bases.jl:98-139): TTR, write v_{j+1} with its
        // Gram row, the loss check on the device (post LAN_FIN sets SC_REDO per factor),
        // then the MGS redo of step j as gated launches: blocks of factors whose flag is
        // clear return at once.  No host round trip, so the step can be swept.
        RUN(TCLS_PASS1, 2, launch_lan_l1_plain(dc->df, nf, a, s), "lan_l1_plain");
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, 1, dc->npart, s), "reduce");
        RUN(TCLS_PASS2, 2, launch_lan_l2(dc->df, nf, a, s), "lan_l2");
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 2, 1, dc->npart, s), "reduce");
        RUN(TCLS_RED, 2, launch_post(dc->df, nf, a, POST_LAN, 0, 1, s), "post");
        if (dc->fin_d && j + 1 <= D1_JMAX) {
            RUN(TCLS_FIN, 2, launch_fin_d(dc->df, nf, a, 1, s), "fin_d");
            RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, j + 3, dc->ntiles, s), "reduce");
        } else {
            RUN(TCLS_FIN, 2, launch_lan_finalize(dc->df, nf, a, s), "lan_finalize");
            RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, j + 3, dc->npart, s), "reduce");
        }
        RUN(TCLS_RED, 2, launch_post(dc->df, nf, a, POST_LAN_FIN, 1, 0, s), "post");
        KArgs g = a;
        g.gate = 1;
        RUN(TCLS_PASS1, 2, launch_arn_a1_plain(dc->df, nf, g, s), "arn_a1_plain");
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 1, j + 1, dc->npart, s, 1), "reduce");
        RUN(TCLS_PASS2, 2, launch_arn_a2(dc->df, nf, g, s), "arn_a2");
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 2, 2 * j + 4, dc->npart, s, 1), "reduce");
        RUN(TCLS_RED, 2, launch_post(dc->df, nf, g, POST_ARN, 0, 0, s), "post");
        RUN(TCLS_FIN, 2, launch_arn_finalize(dc->df, nf, g, s), "arn_finalize");
        RUN(TCLS_RED, 2, launch_reduce(dc->df, nf, 3, j + 3, dc->npart, s, 1), "reduce");
        RUN(TCLS_RED, 2, launch_post(dc->df, nf, g, POST_ARN_FIN, 0, 0, s), "post");
        // the record is final only after the gated redo: one ungated launch mirrors it to
        // the host (the exchange of a LanczosReorth handle waits on an event instead)
        if (hsig) RUN(TCLS_RED, 2, launch_post(dc->df, nf, ax, POST_SIGNAL, 0, 0, s), "post_signal");
        dc->pending = false;
    }
    dc->last_j = j;
    dc->jnext = j + 1;
    return TK_OK;
}

tk_status tk_decomp_step(tk_decomp* dc, int j, double* rec_out) { TK_API_BEGIN
    CHECKARG(dc, "NULL decomp");
    if (dc->failed) return fail(TK_ERR_STATE, "an earlier step of this decomposition failed");
    if (!dc->inited) return fail(TK_ERR_STATE, "tk_decomp_init not called");
    if (j != dc->jnext) return fail(TK_ERR_STATE, "step %d requested, next step is %d", j, dc->jnext);
    if (j >= dc->kmax) return fail(TK_ERR_ARG, "step %d >= kmax %d", j, dc->kmax);
    HIPCHK(hipSetDevice(dc->ctx->device));
    HpScope hp_step(HP_STEP);
    const int prev_bk = dc->bk_j;
    const unsigned long long prev_seq = dc->bk_args.seq, prev_xval = dc->bk_args.xval;
#if TK_TEST_BUILD
    tk_status st = j == dc->fail_step ? fail(TK_ERR_HIP, "step %d: injected failure (TKHIP_TEST_FAIL_STEP)", j)
                                      : step_impl(dc, j, rec_out);
#else
    tk_status st = step_impl(dc, j, rec_out);
#endif
    if (st) {
        // the exchange stream only ever waits for signal counts of steps that were fully
        // enqueued, so a failed step cannot leave it blocked (destroy stays safe)
        dc->failed = true;
        return st;
    }
    HpScope hp_bk(HP_BK);
    if (dc->bk_j == j) {
        // one sweep: this launch carried step j-1's bookkeeping (its record is complete);
        // step j's own waits for the next launch unless the caller wants it now
        if (prev_bk == j - 1 && prev_bk >= 0) complete_step(dc, prev_bk, prev_seq, prev_xval);
        if (rec_out || !dc->bk_fold) {
            st = bk_flush(dc);
            if (st) return st;
        }
    } else {
        complete_step(dc, j, dc->seq, dc->cur_xval);
    }
    if (dc->recv != dc->rec) {
        // canonical: slots <= j are written on every rank now; full groups go out
        for (const XSched::Range& r : dc->xs.step_done(j)) {
            st = xsend(dc, r);
            if (st) return st;
        }
        if (rec_out) {
            st = need_slots(dc, j + 1);
            if (st) return st;
        }
    }
    return copy_slot(dc, j + 1, rec_out);
    TK_API_END
}

tk_status tk_decomp_sweep(tk_decomp* dc, int j0, int j1) { TK_API_BEGIN
    CHECKARG(dc, "NULL decomp");
    // one event pair brackets the whole sweep (events between the steps would idle the
    // GPU for their fences and inflate the very time they measure)
    Timer sweep_timer(dc->ctx, TCLS_SWEEP, 1);
    dc->in_sweep = true;
    tk_status st = TK_OK;
    for (int j = j0; j < j1 && st == TK_OK; ++j) st = tk_decomp_step(dc, j, nullptr);
    dc->in_sweep = false;
    if (st == TK_OK) st = bk_flush(dc);
    if (st == TK_OK) st = join_groups(dc);
    if (st == TK_OK) st = need_slots(dc, dc->jnext);
    return st;
    TK_API_END
}

tk_status tk_decomp_flush(tk_decomp* dc, double* rec_out) { TK_API_BEGIN
    CHECKARG(dc, "NULL decomp");
    if (dc->failed) return fail(TK_ERR_STATE, "an earlier step of this decomposition failed");
    HIPCHK(hipSetDevice(dc->ctx->device));
    {
        tk_status st0 = bk_flush(dc);
        if (st0 == TK_OK) st0 = need_slots(dc, dc->jnext);   // every issued step's slot first
        if (st0) return st0;
    }
    const int slot = dc->kmax + 1;
    const bool multi = dc->recv != dc->rec;
    if (!dc->pending) {
        if (rec_out) {
            tk_status st = clear_slot(dc, slot);
            if (st == TK_OK && multi) st = exchange_range(dc, slot, slot);
            if (st) return st;
            return copy_slot(dc, slot, rec_out);
        }
        return TK_OK;
    }
    tk_status st = slot_guard(dc, slot);
    if (st) return st;
    KArgs a = base_args(dc, dc->last_j, slot);
    st = finalize_pending(dc, a);
    if (st) return st;
    dc->pending = false;
    if (multi) {
        st = exchange_range(dc, slot, slot);
        if (st) return st;
    }
    return copy_slot(dc, slot, rec_out);
    TK_API_END
}

// TKHIP_TEST_XCH_STALL: release the exchange stream held at the stalled range (tests)
static void release_stall(tk_decomp* dc) {
    if (!dc->stallw) return;
    const unsigned long long v = dc->stall_v + 1;
    hipMemcpy(dc->stallw, &v, sizeof v, hipMemcpyHostToDevice);
}

tk_status tk_decomp_records(tk_decomp* dc, int s0, int s1, double* out) { TK_API_BEGIN
    CHECKARG(dc && out, "NULL argument");
    CHECKARG(s0 >= 0 && s1 <= dc->kmax + 2 && s0 <= s1, "slot range");
    tk_ctx* c = dc->ctx;
    HIPCHK(hipSetDevice(c->device));
    const size_t per = (size_t)dc->d_total * dc->m;
    if (s1 == s0) return TK_OK;
    if (dc->recv != dc->rec) {
        // the step slots up to s1-1 go out now if their group has not (the flush slot went
        // out with its flush); canonical on every rank
        if (!dc->failed) {
            tk_status st = need_slots(dc, std::min(s1 - 1, dc->jnext));
            if (st) return st;
        }
    } else if (dc->bk_j >= 0 && dc->bk_j + 1 >= s0 && dc->bk_j + 1 < s1 && !dc->failed) {
        tk_status st = bk_flush(dc);
        if (st) return st;
    }
    bool hosted = dc->hdone != nullptr;
    for (int sl = s0; sl < s1 && hosted; ++sl) hosted = dc->slot_seq[sl] != 0;
    if (hosted) {
        // wait for the steps that wrote these slots only (later steps may be queued or
        // running), then read their records from host-mapped memory
        Deadline dl(ctx_wait_limit(c));
        for (int sl = s0; sl < s1; ++sl) {
            const unsigned long long want = dc->slot_seq[sl];
            const unsigned long long* w = dc->hdone + (size_t)sl * dc->nf;
            for (int f = 0; f < dc->nf; ++f) {
                long spins = 0;
                while (__atomic_load_n(w + f, __ATOMIC_ACQUIRE) < want) {
                    TK_POLL_RELAX();
                    if (++spins % 4096 == 0) {
                        // the device may have failed: surface its error instead of spinning (both
                        // factor-group streams: the records are late only if neither runs)
                        hipError_t e = hipStreamQuery(c->stream);
                        for (int g = 1; e == hipSuccess && g < dc->ngr; ++g) e = hipStreamQuery(grp_stream(dc, g));
                        if (e != hipSuccess && e != hipErrorNotReady)
                            return fail(TK_ERR_HIP, "waiting for step records: %s", hipGetErrorString(e));
                        if (e == hipSuccess && __atomic_load_n(w + f, __ATOMIC_ACQUIRE) < want)
                            return fail(TK_ERR_STATE, "step records of slot %d never arrived", sl);
                        // (a deadline where a peer could hold the queue back, or TKHIP_LOCAL_WAIT_S)
                        if (dl.over())
                            return fail(TK_ERR_HIP, "step records of slot %d: not complete after %.0f s", sl, dl.lim);
                    }
                }
            }
        }
        memcpy(out, dc->hrec + (size_t)s0 * per, (s1 - s0) * per * sizeof(double));
        return werr_check(c, "tk_decomp_records");
    }
    bool xhosted = dc->xdone != nullptr;
    for (int sl = s0; sl < s1 && xhosted; ++sl) xhosted = dc->xslot_seq[sl] != 0;
    if (xhosted) {
        // multi-rank: wait for the exchange stream's mirror of each slot (host-mapped words)
        Deadline dl;
        for (int sl = s0; sl < s1; ++sl) {
            const unsigned long long want = dc->xslot_seq[sl];
            long spins = 0;
            while (__atomic_load_n(dc->xdone + sl, __ATOMIC_ACQUIRE) < want) {
                TK_POLL_RELAX();
                if (++spins % 4096 == 0) {
                    hipError_t e = hipStreamQuery(c->xstream);
                    if (e != hipSuccess && e != hipErrorNotReady)
                        return fail(TK_ERR_HIP, "waiting for exchanged records: %s", hipGetErrorString(e));
                    if (e == hipSuccess && __atomic_load_n(dc->xdone + sl, __ATOMIC_ACQUIRE) < want)
                        return fail(TK_ERR_STATE, "exchanged records of slot %d never arrived", sl);
                    if (dl.elapsed() > dl.lim) {
                        const tk_status st = wait_expired(c, "records exchange", sl);
                        release_stall(dc);
                        return st;
                    }
                }
            }
        }
        memcpy(out, dc->hrec + (size_t)s0 * per, (s1 - s0) * per * sizeof(double));
        return werr_check(c, "tk_decomp_records");
    }
    if (dc->cstream && dc->recv != dc->rec) {
        // multi-rank: the slots are final once the exchange of the last one SENT in this
        // sequence has run (exchanges run in slot order on the exchange stream); copy on a
        // stream of its own.  A slot past xs.sent (e.g. a flush slot no flush filled) has no
        // exchange: waiting on its never-recorded event returned at once and the copy could
        // overtake the last real exchange (found by the multi-process test, round 6)
        const int w = std::min(s1 - 1, dc->xs.sent);
        if (w >= s0) {
            tk_status st = event_bounded(c, dc->ev_x[dc->xev[w]], "records exchange", w);
            if (st) {
                release_stall(dc);
                return st;
            }
        }
        HIPCHK(hipMemcpyAsync(out, dc->recv + s0 * per, (s1 - s0) * per * sizeof(double), hipMemcpyDeviceToHost,
                              dc->cstream));
        HIPCHK(hipStreamSynchronize(dc->cstream));
        return werr_check(c, "tk_decomp_records");
    }
    if (dc->recv != dc->rec) {
        tk_status st = sync_bounded(c, c->xstream, "records exchange", s1 - 1);
        if (st) return st;
    }
    GJOIN(dc);
    HIPCHK(hipMemcpyAsync(out, dc->recv + s0 * per, (s1 - s0) * per * sizeof(double), hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return werr_check(c, "tk_decomp_records");
    TK_API_END
}

tk_status tk_decomp_get_basis(tk_decomp* dc, int f, int c0, int nc, double* out) { TK_API_BEGIN
    CHECKARG(dc && out, "NULL argument");
    CHECKARG(f >= 0 && f < dc->nf, "factor out of range");
    CHECKARG(c0 >= 0 && nc >= 0 && c0 + nc <= dc->kmax + 1, "column range");
    HIPCHK(hipSetDevice(dc->ctx->device));
    GJOIN(dc);
    // (one-sweep Arnoldi after an even step: column last_j is still in DFac::E; the flush
    // stores it with the pending column)
    const bool in_e = (dc->method == TK_ARNOLDI || dc->method == TK_LANCZOS) && dc->onesweep && !dc->sl &&
                      dc->last_j <= ARN_D1_JMAX && !(dc->last_j & 1);
    if (dc->pending && nc > 0 && c0 + nc - 1 >= dc->last_j + (in_e ? 0 : 1)) {
        // (as tk_decomp_gram: a one-rank read must not start collectives its peers do not join)
        if (dc->recv != dc->rec && dc->ctx->nranks > 1)
            return fail(TK_ERR_STATE, "tk_decomp_get_basis: column %d is pending; call tk_decomp_flush on every rank first",
                        dc->last_j + 1);
        tk_status st = tk_decomp_flush(dc, nullptr);
        if (st) return st;
    }
    if (nc == 0) return TK_OK;
    const DFac& d = dc->hf[f];
    hipStream_t s = dc->ctx->stream;
    // gather GCH columns at a time from the tile-major basis into a persistent scratch
    const int GCH = 8;
    if (!dc->scratch) {
        HIPCHK(hipMalloc((void**)&dc->scratch, (size_t)dc->n * GCH * sizeof(double)));
    }
    for (int cc = 0; cc < nc; cc += GCH) {
        const int m = std::min(GCH, nc - cc);
        launch_get_cols(d.V, dc->n, dc->kmax, c0 + cc, m, dc->scratch, dc->sl ? 1 : 0, s);
        LAUNCHCHK("get_cols");
        HIPCHK(hipStreamSynchronize(s));
        HIPCHK(hipMemcpy(out + (size_t)cc * dc->n, dc->scratch, (size_t)dc->n * m * sizeof(double),
                         hipMemcpyDeviceToHost));
    }
    return werr_check(dc->ctx, "tk_decomp_get_basis");
    TK_API_END
}

// wait (host spin on the mapped sequence word) for the Gram whose mirror publishes `want`
static tk_status gram_wait(tk_decomp* dc, hipStream_t s, unsigned long long want) {
    tk_ctx* c = dc->ctx;
    long spins = 0;
    Deadline dl(ctx_wait_limit(c));
    while (__atomic_load_n(dc->gram_done, __ATOMIC_ACQUIRE) < want) {
        TK_POLL_RELAX();
        if (++spins % 4096 == 0) {
            hipError_t e = hipStreamQuery(s);
            if (e != hipSuccess && e != hipErrorNotReady) return fail(TK_ERR_HIP, "tk_decomp_gram: %s", hipGetErrorString(e));
            if (e == hipSuccess && __atomic_load_n(dc->gram_done, __ATOMIC_ACQUIRE) < want)
                return fail(TK_ERR_STATE, "tk_decomp_gram: the result never arrived");
            if (dl.over())
                return fail(TK_ERR_HIP, "tk_decomp_gram: not complete after %.0f s", dl.lim);
        }
    }
    return werr_check(c, "tk_decomp_gram");
}

tk_status tk_decomp_gram(tk_decomp* dc, int f, int k, double* G) { TK_API_BEGIN
    CHECKARG(dc, "NULL argument");
    CHECKARG(f >= 0 && f < dc->nf, "factor out of range");
    CHECKARG(k >= 1 && k <= 64 && k <= dc->kmax + 1, "k out of range [1, min(64, kmax+1)]");
    tk_ctx* c = dc->ctx;
    HIPCHK(hipSetDevice(c->device));
    GJOIN(dc);
    if (dc->failed) return fail(TK_ERR_STATE, "an earlier step of this decomposition failed");
    if (f == 0 && dc->ahead_k >= k && dc->gram_host) {
        // launched ahead (tk_decomp_gram_ahead) over these columns: read its leading block
        if (!G) return TK_OK;
        tk_status st = gram_wait(dc, c->stream, dc->ahead_want);
        if (st) return st;
        std::vector<double> full((size_t)dc->ahead_k * dc->ahead_k);
        gram_unpack(dc->ahead_k, dc->gram_host, full.data());
        for (int j = 0; j < k; ++j)
            for (int i = 0; i < k; ++i) G[(size_t)j * k + i] = full[(size_t)j * dc->ahead_k + i];
        return TK_OK;
    }
    dc->ahead_k = 0;   // (this launch's mirror replaces the one launched ahead)
    // every column the product reads must be in V: flush a pending (or column-buffered) one
    const bool in_e = (dc->method == TK_ARNOLDI || dc->method == TK_LANCZOS) && dc->onesweep && !dc->sl &&
                      dc->last_j <= ARN_D1_JMAX && !(dc->last_j & 1);
    if (dc->pending && k - 1 >= dc->last_j + (in_e ? 0 : 1)) {
        // the flush starts record all-reduces (need_slots, the flush slot): with peers, only a
        // call every rank makes may start them, and the Gram is one rank's -- the caller
        // flushes on every rank first (tkamd.solver._fill_deferred_orthogonality)
        if (dc->recv != dc->rec && c->nranks > 1)
            return fail(TK_ERR_STATE, "tk_decomp_gram: column %d is pending; call tk_decomp_flush on every rank first",
                        dc->last_j + 1);
        tk_status st = tk_decomp_flush(dc, nullptr);
        if (st) return st;
    }
    if (!dc->gram_scr) HIPCHK(hipMalloc((void**)&dc->gram_scr, gram_scratch_doubles(dc->ntiles) * sizeof(double)));
    // after everything enqueued so far (the steps that wrote columns < k): on the compute
    // stream itself by default -- run beside the end-of-solve V*Y the two kernels took longer
    // together than one after the other, and the two cross-stream event hand-offs of the side
    // stream cost the tracked factor's rank ~100 us per solve at one factor per GPU
    // (TKHIP_GRAM_STREAM=side keeps the side stream for experiments)
    static const bool side = [] {
        const char* e = getenv("TKHIP_GRAM_STREAM");
        return e && !strcmp(e, "side");
    }();
    hipStream_t s = side ? c->gstream : c->stream;
    if (side) {
        HIPCHK(hipEventRecord(dc->gev_in, c->stream));
        HIPCHK(hipStreamWaitEvent(s, dc->gev_in, 0));
    }
    {
        Timer tm(c, TCLS_GRAM, 1, s);
        KArgs a = base_args(dc, 0, 0);
        launch_gram(dc->df, f, a, k, dc->gram_scr, s);
    }
    LAUNCHCHK("gram");
    if (side) {
        HIPCHK(hipEventRecord(dc->gev_done, s));
        dc->gram_inflight = true;
    }
    if (!G) return TK_OK;
    const int nv = gram_values(k);
    std::vector<double> vbuf;
    const double* v = dc->gram_host;
    const double* res = dc->gram_scr + gram_result_offset(dc->ntiles, k);
    if (v) {
        const unsigned long long want = ++dc->gram_seq;
        launch_mirror_records(res, dc->gram_host, nv, dc->gram_done, 1, want, s);
        LAUNCHCHK("gram mirror");
        tk_status st = gram_wait(dc, s, want);
        if (st) return st;
    } else {
        vbuf.resize(nv);
        HIPCHK(hipMemcpyAsync(vbuf.data(), res, nv * sizeof(double), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        tk_status sw = werr_check(c, "tk_decomp_gram");
        if (sw) return sw;
        v = vbuf.data();
    }
    gram_unpack(k, v, G);
    return TK_OK;
    TK_API_END
}

tk_status tk_decomp_gram_ahead(tk_decomp* dc, int* k_out) { TK_API_BEGIN
    CHECKARG(dc && k_out, "NULL argument");
    *k_out = 0;
    tk_ctx* c = dc->ctx;
    // only the rank holding global factor 0 (not a replica) of a deferred-Gram handle, with
    // the host mirror available, and never twice per sequence
    static const bool off = [] {   // TKHIP_GRAM_AHEAD=0: the Gram waits for the caller (A/B, tests)
        const char* e = getenv("TKHIP_GRAM_AHEAD");
        return e && e[0] == '0';
    }();
    if (off || !dc->gram_deferred || dc->foff != 0 || dc->nf <= 0 || dc->zrec || !dc->gram_host || dc->failed ||
        !dc->inited || dc->ahead_k > 0)
        return TK_OK;
    // written columns only (no flush: it would start record exchanges on one rank)
    const bool in_e = (dc->method == TK_ARNOLDI || dc->method == TK_LANCZOS) && dc->onesweep && !dc->sl &&
                      dc->last_j <= ARN_D1_JMAX && !(dc->last_j & 1);
    int k = dc->pending ? dc->last_j + (in_e ? 0 : 1) : dc->jnext + 1;
    k = std::min(std::min(k, 64), dc->kmax + 1);
    if (k < 2) return TK_OK;
    HIPCHK(hipSetDevice(c->device));
    // the last step's deferred bookkeeping (its record, host mirror and exchange signal) goes
    // first: behind the SYRK, the final iteration's record -- and with peers that slot's
    // all-reduce -- would wait for the whole Gram.  Local: no collective
    tk_status st = bk_flush(dc);
    if (st) return st;
    GJOIN(dc);
    if (!dc->gram_scr) HIPCHK(hipMalloc((void**)&dc->gram_scr, gram_scratch_doubles(dc->ntiles) * sizeof(double)));
    hipStream_t s = c->stream;
    {
        Timer tm(c, TCLS_GRAM, 1, s);
        KArgs a = base_args(dc, 0, 0);
        launch_gram(dc->df, 0, a, k, dc->gram_scr, s);
    }
    LAUNCHCHK("gram ahead");
    const unsigned long long want = ++dc->gram_seq;
    launch_mirror_records(dc->gram_scr + gram_result_offset(dc->ntiles, k), dc->gram_host, gram_values(k),
                          dc->gram_done, 1, want, s);
    LAUNCHCHK("gram ahead mirror");
    dc->ahead_k = k;
    dc->ahead_want = want;
    *k_out = k;
    return TK_OK;
    TK_API_END
}

tk_status tk_decomp_basis_mul(tk_decomp* dc, int k, int t, const double* Y, double* X) { TK_API_BEGIN
    CHECKARG(dc && Y, "NULL argument");
    CHECKARG(k >= 1 && k <= dc->kmax + 1 && t >= 1, "bad k/t");
    tk_ctx* c = dc->ctx;
    HIPCHK(hipSetDevice(c->device));
    GJOIN(dc);
    if (dc->failed) return fail(TK_ERR_STATE, "an earlier step of this decomposition failed");
    {
        tk_status st0 = bk_flush(dc);
        if (st0 == TK_OK && dc->pending) st0 = need_slots(dc, dc->jnext);   // as tk_decomp_flush
        if (st0) return st0;
    }
    // a pending column is finalized first; for Arnoldi with the one-tile flush kernel it is
    // done in the same launch as V*Y (each basis tile streamed once for both)
    const int jl = dc->last_j;
    const char* nofuse = getenv("TKHIP_NO_FUSED_FLUSH");
    // (the one-sweep Lanczos' pending column too: its flush reads the same register row)
    const bool lan1 = dc->method == TK_LANCZOS && dc->onesweep && jl <= ARN_D1_JMAX;
    const bool fuse = dc->pending && (dc->method == TK_ARNOLDI || lan1) && dc->fin_d && jl + 1 <= D1_JMAX &&
                      k <= jl + 1 && !(nofuse && nofuse[0] == '1');
    const int ldy = fuse ? 64 : k;   // fused: Y_s columns zero-padded to the register row's width
    if (dc->pending && !fuse) {
        tk_status st = tk_decomp_flush(dc, nullptr);
        if (st) return st;
    }
    const size_t ny = (size_t)dc->nf * ldy * t, nx = (size_t)dc->nf * dc->ld * t;
    if (ny > dc->ycap) {
        if (dc->Ydev) hipFree(dc->Ydev);
        dc->Ydev = nullptr;
        HIPCHK(hipMalloc(&dc->Ydev, ny * sizeof(double)));
        dc->ycap = ny;
    }
    if (nx > dc->xcap) {
        if (dc->Xdev) hipFree(dc->Xdev);
        dc->Xdev = nullptr;
        HIPCHK(hipMalloc(&dc->Xdev, nx * sizeof(double)));
        dc->xcap = nx;
    }
    hipStream_t s = c->stream;
    if (fuse) {
        // Y_s columns zero-padded to ldy rows (tiny: nf * t * 64 doubles); a pageable-source
        // copy is staged before hipMemcpyAsync returns, as for the caller's Y below
        std::vector<double> yp(ny, 0.0);
        for (int f = 0; f < dc->nf; ++f)
            for (int q = 0; q < t; ++q)
                memcpy(&yp[((size_t)f * t + q) * ldy], Y + ((size_t)f * t + q) * k, (size_t)k * sizeof(double));
        HIPCHK(hipMemcpyAsync(dc->Ydev, yp.data(), ny * sizeof(double), hipMemcpyHostToDevice, s));
    } else {
        HIPCHK(hipMemcpyAsync(dc->Ydev, Y, ny * sizeof(double), hipMemcpyHostToDevice, s));
    }
    if (fuse) {
        const int slot = dc->kmax + 1;
        tk_status st = slot_guard(dc, slot);
        if (st) return st;
        KArgs a = base_args(dc, jl, slot);
        KArgs f = a;
        if (dc->onesweep && jl <= ARN_D1_JMAX) {   // as finalize_pending
            f.ubuf = (jl & 1) ? 0 : 1;
            f.ecol = (dc->sl || (jl & 1)) ? -1 : jl;
        }
        RUN(TCLS_VY, 1, launch_fin_vy(dc->df, dc->nf, f, dc->Ydev, dc->Xdev, ldy, t, lan1 ? 2 : 0, s), "fin_vy");
        if (lan1) {
            RUN(TCLS_RED, 2, launch_reduce(dc->df, dc->nf, 1, jl + 3, dc->ntiles, s), "reduce");
            RUN(TCLS_RED, 2, launch_post(dc->df, dc->nf, a, POST_LAN_FIN, 0, 1, s), "post");
        } else {
            RUN(TCLS_RED, 2, launch_reduce(dc->df, dc->nf, 3, jl + 3, dc->ntiles, s), "reduce");
            RUN(TCLS_RED, 2, launch_post(dc->df, dc->nf, a, POST_ARN_FIN, 0, 1, s), "post");
        }
        dc->pending = false;
        if (dc->recv != dc->rec) {
            st = exchange_range(dc, slot, slot);
            if (st) return st;
        }
    } else {
        KArgs a = base_args(dc, 0, 0);
        RUN(TCLS_VY, 1, launch_basis_mul(dc->df, dc->nf, a, dc->Ydev, dc->Xdev, k, t, s), "basis_mul");
    }
    if (X) {
        // device X_s is tile-major (256-row tiles, each tile's t columns contiguous): copy
        // and reorder to column-major n x t
        HIPCHK(hipStreamSynchronize(s));
        std::vector<double> tmp((size_t)dc->ld * t);
        for (int f = 0; f < dc->nf; ++f) {
            HIPCHK(hipMemcpy(tmp.data(), dc->Xdev + (size_t)f * dc->ld * t, tmp.size() * sizeof(double),
                             hipMemcpyDeviceToHost));
            double* Xf = X + (size_t)f * dc->n * t;
            for (int q = 0; q < t; ++q)
                for (int64_t r = 0; r < dc->n; ++r)
                    Xf[(size_t)q * dc->n + r] = tmp[(size_t)(r >> 8) * 256 * t + (size_t)q * 256 + (r & 255)];
        }
        return werr_check(c, "tk_decomp_basis_mul");
    }
    return TK_OK;
    TK_API_END
}

tk_status tk_timing_enable(tk_ctx* c, int on) { TK_API_BEGIN
    CHECKARG(c, "NULL ctx");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    drain_timers(c);
    for (int k = 0; k < TCLS_N; ++k) {
        c->ms[k] = 0.0;
        c->cnt[k] = 0;
    }
    c->timing = on;
    return TK_OK;
    TK_API_END
}

tk_status tk_timing_read(tk_ctx* c, int cls, double* total_ms, long* launches) { TK_API_BEGIN
    CHECKARG(c && total_ms && launches, "NULL argument");
    CHECKARG(cls >= 0 && cls < TCLS_N, "timing class out of range");
    HIPCHK(hipSetDevice(c->device));
    drain_timers(c);
    *total_ms = c->ms[cls];
    *launches = c->cnt[cls];
    return TK_OK;
    TK_API_END
}

}  // extern "C"
