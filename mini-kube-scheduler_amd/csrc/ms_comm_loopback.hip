// ms_comm_loopback.hip — TEST-ONLY in-process communicator for ms_comm.cpp
// (see ms_comm_loopback.h). Built only by `make comm-loopback` into
// libminisched_gpu_loopback.so; the product library links RCCL instead.
#include "ms_comm_loopback.h"

#include <atomic>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr int kMaxRanks = 16;
constexpr auto kJoinTimeout = std::chrono::seconds(120);

struct Post {
    int kind = 0;  // 1 reduce-scatter, 2 all-gather, 3 all-to-all
    const void *send = nullptr;
    void *recv = nullptr;
    size_t count = 0;
    ncclDataType_t dt = ncclUint8;
    ncclRedOp_t op = ncclSum;
};

struct Group {
    int world = 0;
    bool solo = false;  // MS_LB_SOLO: one rank of `world` stands alone (per-rank probes)
    std::mutex mu;
    std::condition_variable cv;
    int joined = 0, left = 0;
    int arrived = 0;
    uint64_t gen = 0;  // barrier generation
    Post post[kMaxRanks];
    hipEvent_t ev_send[kMaxRanks] = {}, ev_done[kMaxRanks] = {};
};

struct Comm {
    std::shared_ptr<Group> g;
    int rank = 0;
};

std::mutex g_reg_mu;
std::map<std::string, std::shared_ptr<Group>> g_reg;  // id bytes -> group being formed
std::atomic<unsigned long long> g_issued{0};
std::atomic<unsigned long long> g_id_counter{1};

// Generation barrier over the group's ranks; false on timeout.
bool barrier(Group &g) {
    if (g.solo) return true;
    std::unique_lock<std::mutex> lk(g.mu);
    const uint64_t my = g.gen;
    if (++g.arrived == g.world) {
        g.arrived = 0;
        ++g.gen;
        g.cv.notify_all();
        return true;
    }
    return g.cv.wait_for(lk, kJoinTimeout, [&] { return g.gen != my; });
}

size_t dt_size(ncclDataType_t d) {
    switch (d) {
        case ncclUint8: case ncclInt8: return 1;
        case ncclUint32: case ncclInt32: return 4;
        case ncclUint64: case ncclInt64: return 8;
        default: return 0;
    }
}

struct Srcs {
    const void *p[kMaxRanks];
};

// out[i] = max over the G ranks of src_j[base + i] (unsigned element-wise MAX)
template <typename T>
__global__ void k_lb_max(Srcs s, int G, size_t base, size_t n, T *out) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        T m = static_cast<const T *>(s.p[0])[base + i];
        for (int j = 1; j < G; ++j) {
            const T v = static_cast<const T *>(s.p[j])[base + i];
            m = v > m ? v : m;
        }
        out[i] = m;
    }
}

template <typename T>
hipError_t launch_max(const Srcs &s, int G, size_t base, size_t n, void *out, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_lb_max<T>, dim3(blocks), dim3(256), 0, st, s, G, base, n, static_cast<T *>(out));
    return hipGetLastError();
}

// One collective on rank r: post, barrier, wait for every rank's send event,
// combine this rank's output, barrier, wait for every rank's done event.
// Solo (MS_LB_SOLO, per-rank probes): every other rank is taken to have sent
// this rank's own buffer, so a reduce-scatter combines G copies of its block r
// (the G-way MAX a real rank computes), an all-gather writes its block into all
// G slots, an all-to-all its block r into all G; the work and bytes of one rank
// of a G-rank collective, without the others.
ncclResult_t collective(Comm *c, const Post &p, hipStream_t st) {
    Group &g = *c->g;
    const int r = c->rank, G = g.world;
    if (g.solo) {
        const size_t es = dt_size(p.dt), bytes = p.count * es;
        hipError_t e = hipSuccess;
        if (p.kind == 1) {
            Srcs s{};
            for (int j = 0; j < G; ++j) s.p[j] = p.send;
            const size_t base = (size_t)r * p.count;
            if (es == 1) e = launch_max<uint8_t>(s, G, base, p.count, p.recv, st);
            else if (es == 4) e = launch_max<uint32_t>(s, G, base, p.count, p.recv, st);
            else e = launch_max<unsigned long long>(s, G, base, p.count, p.recv, st);
        } else {
            const char *src = static_cast<const char *>(p.send) + (p.kind == 3 ? (size_t)r * bytes : 0);
            for (int j = 0; j < G && e == hipSuccess; ++j) {
                char *dst = static_cast<char *>(p.recv) + (size_t)j * bytes;
                if (dst != src && bytes) e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, st);
            }
        }
        if (e != hipSuccess) return ncclUnhandledCudaError;
        g_issued.fetch_add(1);
        return ncclSuccess;
    }
    if (hipEventRecord(g.ev_send[r], st) != hipSuccess) return ncclUnhandledCudaError;
    g.post[r] = p;
    if (!barrier(g)) return ncclSystemError;  // a rank never issued this collective
    for (int j = 0; j < G; ++j) {  // every rank issues the same sequence (as RCCL requires)
        const Post &q = g.post[j];
        if (q.kind != p.kind || q.count != p.count || q.dt != p.dt || q.op != p.op) return ncclInvalidUsage;
    }
    for (int j = 0; j < G; ++j)
        if (j != r && hipStreamWaitEvent(st, g.ev_send[j], 0) != hipSuccess) return ncclUnhandledCudaError;
    const size_t es = dt_size(p.dt);
    hipError_t e = hipSuccess;
    if (p.kind == 1) {  // reduce-scatter: rank r's block r of every send buffer
        Srcs s{};
        for (int j = 0; j < G; ++j) s.p[j] = g.post[j].send;
        const size_t base = (size_t)r * p.count;
        if (es == 1) e = launch_max<uint8_t>(s, G, base, p.count, p.recv, st);
        else if (es == 4) e = launch_max<uint32_t>(s, G, base, p.count, p.recv, st);
        else e = launch_max<unsigned long long>(s, G, base, p.count, p.recv, st);
    } else if (p.kind == 2) {  // all-gather: rank j's send buffer into block j of this rank's recv
        const size_t bytes = p.count * es;
        for (int j = 0; j < G && e == hipSuccess; ++j) {
            char *dst = static_cast<char *>(p.recv) + (size_t)j * bytes;
            if (dst != g.post[j].send && bytes)  // (in place: this rank's own block is already there)
                e = hipMemcpyAsync(dst, g.post[j].send, bytes, hipMemcpyDeviceToDevice, st);
        }
    } else {  // all-to-all: block r of rank j's send buffer into block j of this rank's recv
        const size_t bytes = p.count * es;
        for (int j = 0; j < G && e == hipSuccess; ++j)
            if (bytes)
                e = hipMemcpyAsync(static_cast<char *>(p.recv) + (size_t)j * bytes,
                                   static_cast<const char *>(g.post[j].send) + (size_t)r * bytes, bytes,
                                   hipMemcpyDeviceToDevice, st);
    }
    if (e != hipSuccess) return ncclUnhandledCudaError;
    if (hipEventRecord(g.ev_done[r], st) != hipSuccess) return ncclUnhandledCudaError;
    if (!barrier(g)) return ncclSystemError;
    for (int j = 0; j < G; ++j)
        if (j != r && hipStreamWaitEvent(st, g.ev_done[j], 0) != hipSuccess) return ncclUnhandledCudaError;
    if (r == 0) g_issued.fetch_add(1);
    return ncclSuccess;
}

}  // namespace

extern "C" {

ncclResult_t lb_ncclGetUniqueId(ncclUniqueId *id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id, 0, sizeof(*id));
    const unsigned long long k = g_id_counter.fetch_add(1);
    const unsigned long long t = (unsigned long long)std::chrono::steady_clock::now().time_since_epoch().count();
    std::memcpy(id->internal, "msloopback", 10);
    std::memcpy(id->internal + 16, &k, sizeof(k));
    std::memcpy(id->internal + 24, &t, sizeof(t));
    return ncclSuccess;
}

ncclResult_t lb_ncclCommInitRank(ncclComm_t *comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    if (const char *solo = getenv("MS_LB_SOLO"); solo && solo[0] == '1') {  // (test / probe builds only)
        auto g = std::make_shared<Group>();
        g->world = nranks;
        g->solo = true;
        if (hipEventCreateWithFlags(&g->ev_send[rank], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g->ev_done[rank], hipEventDisableTiming) != hipSuccess)
            return ncclUnhandledCudaError;
        *comm = reinterpret_cast<ncclComm_t>(new Comm{g, rank});
        return ncclSuccess;
    }
    const std::string key(id.internal, sizeof(id.internal));
    std::shared_ptr<Group> g;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_reg.find(key);
        if (it == g_reg.end()) {
            g = std::make_shared<Group>();
            g->world = nranks;
            g_reg[key] = g;
        } else {
            g = it->second;
        }
    }
    if (g->world != nranks) return ncclInvalidUsage;
    {
        std::lock_guard<std::mutex> lk(g->mu);
        if (g->ev_send[rank]) return ncclInvalidUsage;  // rank joined twice
        if (hipEventCreateWithFlags(&g->ev_send[rank], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&g->ev_done[rank], hipEventDisableTiming) != hipSuccess)
            return ncclUnhandledCudaError;
        ++g->joined;
    }
    if (!barrier(*g)) return ncclSystemError;  // blocks until every rank joined
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        auto it = g_reg.find(key);
        if (it != g_reg.end() && it->second == g) g_reg.erase(it);  // formed: the id may be reused
    }
    Comm *c = new Comm{g, rank};
    *comm = reinterpret_cast<ncclComm_t>(c);
    return ncclSuccess;
}

ncclResult_t lb_ncclCommDestroy(ncclComm_t comm) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    if (!c) return ncclInvalidArgument;
    {
        std::lock_guard<std::mutex> lk(c->g->mu);
        (void)hipEventSynchronize(c->g->ev_done[c->rank]);
        (void)hipEventDestroy(c->g->ev_send[c->rank]);
        (void)hipEventDestroy(c->g->ev_done[c->rank]);
        c->g->ev_send[c->rank] = c->g->ev_done[c->rank] = nullptr;
        ++c->g->left;
    }
    delete c;  // the group goes with its last shared_ptr
    return ncclSuccess;
}

ncclResult_t lb_ncclReduceScatter(const void *sendbuff, void *recvbuff, size_t recvcount, ncclDataType_t datatype,
                                  ncclRedOp_t op, ncclComm_t comm, hipStream_t stream) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    if (!c || op != ncclMax || dt_size(datatype) == 0) return ncclInvalidArgument;  // (the library uses MAX only)
    Post p;
    p.kind = 1;
    p.send = sendbuff;
    p.recv = recvbuff;
    p.count = recvcount;
    p.dt = datatype;
    p.op = op;
    return collective(c, p, stream);
}

ncclResult_t lb_ncclAllGather(const void *sendbuff, void *recvbuff, size_t sendcount, ncclDataType_t datatype,
                              ncclComm_t comm, hipStream_t stream) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    if (!c || dt_size(datatype) == 0) return ncclInvalidArgument;
    Post p;
    p.kind = 2;
    p.send = sendbuff;
    p.recv = recvbuff;
    p.count = sendcount;
    p.dt = datatype;
    return collective(c, p, stream);
}

ncclResult_t lb_ncclAllToAll(const void *sendbuff, void *recvbuff, size_t count, ncclDataType_t datatype,
                             ncclComm_t comm, hipStream_t stream) {
    Comm *c = reinterpret_cast<Comm *>(comm);
    if (!c || dt_size(datatype) == 0) return ncclInvalidArgument;
    Post p;
    p.kind = 3;
    p.send = sendbuff;
    p.recv = recvbuff;
    p.count = count;
    p.dt = datatype;
    return collective(c, p, stream);
}

// Grouping only matters for RCCL's progress; every rank issues the same
// sequence, so the loopback runs each collective as it is called.
ncclResult_t lb_ncclGroupStart() { return ncclSuccess; }
ncclResult_t lb_ncclGroupEnd() { return ncclSuccess; }

const char *lb_ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (loopback)";
        case ncclUnhandledCudaError: return "HIP call failed (loopback)";
        case ncclSystemError: return "rendezvous timed out: a rank did not join or issue the collective (loopback)";
        case ncclInvalidArgument: return "invalid argument (loopback)";
        case ncclInvalidUsage: return "ranks issued different collectives (loopback)";
        default: return "error (loopback)";
    }
}

unsigned long long lb_collectives_issued(void) { return g_issued.load(); }

}  // extern "C"
