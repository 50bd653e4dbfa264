// comm.cpp -- collectives of the distributed solve.
//
// RcclComm: RCCL over xGMI, one process per GPU (production; graph-capturable).
// NullComm: timing stand-in (no peers; see below).
// SimComm:  P ranks as host threads of one process sharing one GPU, exchanging through a
//           shared HBM buffer with host barriers.  It exists so the multi-rank device path
//           can be exercised on a one-GPU box (RCCL refuses two ranks on one device); it is
//           not capturable and not a performance path.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "dev.hpp"

namespace cpk {

namespace {

void nccl_check(ncclResult_t r, const char *what) {
    if (r != ncclSuccess) throw Error(CPK_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
}

struct RcclComm : Comm {
    ncclComm_t c = nullptr;
    ~RcclComm() override {
        if (c) ncclCommDestroy(c);
    }
    void allreduce_sum(double *buf, size_t n, hipStream_t s) override {
        nccl_check(ncclAllReduce(buf, buf, n, ncclDouble, ncclSum, c, s), "ncclAllReduce");
    }
    void allreduce_sum_i64(int64_t *buf, size_t n, hipStream_t s) override {
        nccl_check(ncclAllReduce(buf, buf, n, ncclInt64, ncclSum, c, s), "ncclAllReduce");
    }
    void allgather(const double *send, double *recv, size_t n, hipStream_t s) override {
        nccl_check(ncclAllGather(send, recv, n, ncclDouble, c, s), "ncclAllGather");
    }
    void allreduce_max_i64(int64_t *buf, size_t n, hipStream_t s) override {
        nccl_check(ncclAllReduce(buf, buf, n, ncclInt64, ncclMax, c, s), "ncclAllReduce(max)");
    }
    // host bytes through a device staging buffer, in chunks (RCCL moves device memory only).  The
    // staging buffer is kept across calls (the analysis broadcast makes ~40 of them) and released
    // by release_staging(); it only grows, up to one chunk
    DBuf<char> stage;
    void broadcast_host(void *p, size_t n, int root, hipStream_t s) override {
        if (!n) return;
        int me = 0;
        nccl_check(ncclCommUserRank(c, &me), "ncclCommUserRank");
        constexpr size_t kChunk = size_t(256) << 20;
        if (stage.n < std::min(n, kChunk)) stage.alloc(std::min(n, kChunk));
        char *h = static_cast<char *>(p);
        for (size_t o = 0; o < n; o += kChunk) {
            const size_t k = std::min(kChunk, n - o);
            if (me == root) CPK_HIP(hipMemcpyAsync(stage.p, h + o, k, hipMemcpyHostToDevice, s));
            nccl_check(ncclBroadcast(stage.p, stage.p, k, ncclChar, root, c, s), "ncclBroadcast");
            if (me != root && h) CPK_HIP(hipMemcpyAsync(h + o, stage.p, k, hipMemcpyDeviceToHost, s));
            CPK_HIP(hipStreamSynchronize(s));
        }
    }
    void release_staging() override { stage.release(); }
    bool capturable() const override { return true; }  // the solvers also check the dist_graph option
    int kind() const override { return CPK_COMM_RCCL; }
    int count() const override {
        int n = 0;
        nccl_check(ncclCommCount(c, &n), "ncclCommCount");
        return n;
    }
};

}  // namespace

Comm *make_rccl_comm(int nranks, int rank, const unsigned char *uid) {
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    std::memcpy(&u, uid, 128);
    auto *rc = new RcclComm();
    const ncclResult_t r = ncclCommInitRank(&rc->c, nranks, u, rank);
    if (r != ncclSuccess) {
        delete rc;
        nccl_check(r, "ncclCommInitRank");
    }
    return rc;
}

void rccl_unique_id(unsigned char *uid) {
    ncclUniqueId u;
    nccl_check(ncclGetUniqueId(&u), "ncclGetUniqueId");
    std::memcpy(uid, &u, 128);
}

// ---- timing stand-in ---------------------------------------------------------------------------
// NullComm (diagnostic only, cpk_ctx_create_null): rank `rank` of a P-way partition with no
// peers.  Collectives leave the local contribution in place, so results are meaningless; it
// exists to time one rank's share of a P-way solve on a single GPU (tools/dist_timing.py).
namespace {
struct NullComm : Comm {
    int rank, P;
    NullComm(int r, int p) : rank(r), P(p) {}
    void allreduce_sum(double *, size_t, hipStream_t) override {}
    void allreduce_sum_i64(int64_t *, size_t, hipStream_t) override {}
    void allgather(const double *send, double *recv, size_t n, hipStream_t s) override {
        if (n) CPK_HIP(hipMemcpyAsync(recv + (size_t)rank * n, send, n * sizeof(double), hipMemcpyDeviceToDevice, s));
    }
    void allreduce_max_i64(int64_t *, size_t, hipStream_t) override {}
    void broadcast_host(void *, size_t, int, hipStream_t) override {
        throw Error(CPK_ERR_UNSUPPORTED, "internal: broadcast on the peer-less timing communicator");
    }
    bool capturable() const override { return true; }
    bool has_peers() const override { return false; }
    int kind() const override { return CPK_COMM_NULL; }
    int count() const override { return 1; }  // no peers: the communicator holds this rank only
};
}  // namespace
Comm *make_null_comm(int rank, int nranks) { return new NullComm(rank, nranks); }

// ---- simulated group --------------------------------------------------------------------------
struct SimGroup {
    int P;
    std::mutex mu;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    DBuf<double> shared;  // grown on demand to the largest collective (every rank asks the same n)
    static constexpr size_t kCap0 = size_t(16) << 20;  // doubles
    // each rank's collective count and the last one it entered: a rank that waits in vain names
    // where every rank is (a mismatched collective sequence, or a rank stuck in a device wait)
    std::vector<uint64_t> seq;
    std::vector<std::string> last;
    std::vector<char> host;  // broadcast_host's staging
    int timeout_s = 300;  // CPK_SIM_TIMEOUT_S
    explicit SimGroup(int p) : P(p), seq(p, 0), last(p) {
        if (const char *e = std::getenv("CPK_SIM_TIMEOUT_S")) timeout_s = std::max(1, std::atoi(e));
    }
    void enter(int rank, const char *op, size_t n) {
        std::lock_guard<std::mutex> lk(mu);
        seq[rank]++;
        last[rank] = std::string(op) + "(" + std::to_string(n) + ")";
    }
    void barrier(int rank) {
        std::unique_lock<std::mutex> lk(mu);
        const uint64_t g = gen;
        if (++arrived == P) {
            arrived = 0, gen++;
            cv.notify_all();
            return;
        }
        if (!cv.wait_for(lk, std::chrono::seconds(timeout_s), [&] { return gen != g; })) {
            std::string m = "simulated collective: rank " + std::to_string(rank) + " waited " +
                            std::to_string(timeout_s) + " s;";
            for (int q = 0; q < P; q++) m += " [" + std::to_string(q) + ": #" + std::to_string(seq[q]) + " " + last[q] + "]";
            throw Error(CPK_ERR_RCCL, m);
        }
    }
};

namespace {
struct SimComm : Comm {
    SimGroup *g;
    int rank;
    SimComm(SimGroup *gg, int r) : g(gg), rank(r) {}
    void check(size_t n) const {
        if (n * (size_t)g->P <= g->shared.n) return;
        // every rank of a collective passes the same n: all arrive, rank 0 grows the buffer
        // while the others wait, then all continue with the new one
        g->barrier(rank);
        if (rank == 0) g->shared.alloc(n * (size_t)g->P);
        g->barrier(rank);
    }
    void allreduce_sum(double *buf, size_t n, hipStream_t s) override {
        g->enter(rank, "allreduce_sum", n);
        check(n);
        CPK_HIP(hipMemcpyAsync(g->shared.p + rank * n, buf, n * sizeof(double), hipMemcpyDeviceToDevice, s));
        CPK_HIP(hipStreamSynchronize(s));
        g->barrier(rank);
        launch_sum_slots(s, g->shared.p, g->P, n, buf);
        CPK_HIP(hipStreamSynchronize(s));
        g->barrier(rank);
    }
    void allreduce_sum_i64(int64_t *buf, size_t n, hipStream_t s) override {
        g->enter(rank, "allreduce_sum_i64", n);
        check(n);  // the shared buffer holds 8-byte words: the digits travel as their bits
        int64_t *sh = reinterpret_cast<int64_t *>(g->shared.p);
        CPK_HIP(hipMemcpyAsync(sh + rank * n, buf, n * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
        CPK_HIP(hipStreamSynchronize(s));
        g->barrier(rank);
        launch_sum_slots_i64(s, sh, g->P, n, buf);
        CPK_HIP(hipStreamSynchronize(s));
        g->barrier(rank);
    }
    void allreduce_max_i64(int64_t *buf, size_t n, hipStream_t s) override {
        g->enter(rank, "allreduce_max_i64", n);
        check(n);
        int64_t *sh = reinterpret_cast<int64_t *>(g->shared.p);
        CPK_HIP(hipMemcpyAsync(sh + rank * n, buf, n * sizeof(int64_t), hipMemcpyDeviceToDevice, s));
        CPK_HIP(hipStreamSynchronize(s));
        g->barrier(rank);
        std::vector<int64_t> all(n * (size_t)g->P), mx(n);
        CPK_HIP(hipMemcpyAsync(all.data(), sh, all.size() * sizeof(int64_t), hipMemcpyDeviceToHost, s));
        CPK_HIP(hipStreamSynchronize(s));
        g->barrier(rank);
        for (size_t i = 0; i < n; i++) {
            mx[i] = all[i];
            for (int q = 1; q < g->P; q++) mx[i] = std::max(mx[i], all[(size_t)q * n + i]);
        }
        CPK_HIP(hipMemcpyAsync(buf, mx.data(), n * sizeof(int64_t), hipMemcpyHostToDevice, s));
        CPK_HIP(hipStreamSynchronize(s));
    }
    void allgather(const double *send, double *recv, size_t n, hipStream_t s) override {
        g->enter(rank, "allgather", n);
        check(n);
        if (n) CPK_HIP(hipMemcpyAsync(g->shared.p + rank * n, send, n * sizeof(double), hipMemcpyDeviceToDevice, s));
        CPK_HIP(hipStreamSynchronize(s));
        g->barrier(rank);
        if (n) CPK_HIP(hipMemcpyAsync(recv, g->shared.p, n * g->P * sizeof(double), hipMemcpyDeviceToDevice, s));
        CPK_HIP(hipStreamSynchronize(s));
        g->barrier(rank);
    }
    void broadcast_host(void *p, size_t n, int root, hipStream_t) override {
        g->enter(rank, "broadcast_host", n);
        if (rank == root) g->host.assign(static_cast<char *>(p), static_cast<char *>(p) + n);
        g->barrier(rank);
        if (rank != root && p) std::memcpy(p, g->host.data(), n);
        g->barrier(rank);
        if (rank == root) std::vector<char>().swap(g->host);
    }
    bool capturable() const override { return false; }
    int kind() const override { return CPK_COMM_SIM; }
    int count() const override { return g->P; }
};
}  // namespace

SimGroup *simgroup_create(int nranks) {
    auto *g = new SimGroup(nranks);
    g->shared.alloc(SimGroup::kCap0);
    return g;
}
void simgroup_destroy(SimGroup *g) { delete g; }
Comm *make_sim_comm(SimGroup *g, int rank) { return new SimComm(g, rank); }

}  // namespace cpk
