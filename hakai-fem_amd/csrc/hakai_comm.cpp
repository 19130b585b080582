// hakai_comm.cpp -- multi-GPU interface exchange, one process per GPU over RCCL (xGMI), or an
// in-process group of contexts (tests, several subdomains per device).
//
// Elements are partitioned into contiguous global-id ranges, one per rank (z-slabs for the
// synthetic bars). A node on the boundary between rank r (lower element ids) and r+1 is present
// on both. The reference assembles Q serially in element order (v2/HAKAI_j.jl:669-675), so the
// global order of contributions at such a node is: all of rank r's, then all of rank r+1's.
// Each step, after the element kernel:
//   rank r   sends   P_r  = its own contributions summed in order (3 doubles per node)   -> r+1
//   rank r+1 sends   c_1..c_m, its own contributions one by one (nslot x 3 doubles)      -> r
// and BOTH ranks form Q = ((P_r + c_1) + c_2) + ... , i.e. exactly the single-GPU summation, so an
// N-GPU run is bit-identical to the 1-GPU run. One grouped ncclSend/ncclRecv round per step on a
// second stream; the interior nodal update runs meanwhile and only the interface nodes wait.
// Send buffers alternate by step parity so a receiver may pull step t's data while the sender
// already packs step t+1 (needed by the in-process transport, harmless for RCCL).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "hakai_internal.hpp"

namespace hkc {

struct LocalGroup;

struct Comm {
    int mode = 0;  // 0 RCCL, 1 in-process group
    ncclComm_t nc = nullptr;
    LocalGroup* group = nullptr;
    long long group_key = 0;
    int rank = 0, nranks = 1;
    hipStream_t cs = nullptr;
    hipEvent_t ev_packed[2] = {nullptr, nullptr}, ev_done = nullptr;
    int nslot = 0;
    int n_up = 0, n_dn = 0;          // up: this rank is the lower side (neighbour rank+1); dn: upper side
    int* d_up = nullptr;             // local node ids
    int* d_dn = nullptr;
    double* d_up_sendP[2] = {nullptr, nullptr};  // [n_up][3]
    double* d_up_recvC = nullptr;                // [n_up][nslot][3]
    double* d_dn_sendC[2] = {nullptr, nullptr};  // [n_dn][nslot][3]
    double* d_dn_recvP = nullptr;                // [n_dn][3]
    double* d_saved = nullptr;                   // u_pre of interface nodes [n_up+n_dn][3]
    std::vector<int> h_dn;                       // host copy of d_dn (owner-computed assembly)
    bool pending = false;
    int pending_par = 0;
    // collectives of the multi-GPU contact (hakai_contact.hip) on cs, handed over by events
    hipEvent_t ev_ag_ready = nullptr, ev_ag_done = nullptr;
};

struct LocalGroup {
    int nranks = 0;
    std::vector<hakai_ctx*> ctx;
    int refs = 0;
};

static std::mutex g_groups_mu;
static std::map<long long, LocalGroup*> g_groups;

}  // namespace hkc

using hkc::fail;
using hkc::hip_fail;

#define HIPCHK(x)                                      \
    do {                                               \
        hipError_t _e = (x);                           \
        if (_e != hipSuccess) return hip_fail(_e, #x); \
    } while (0)
#define NCCLCHK(x)                                                                        \
    do {                                                                                  \
        ncclResult_t _r = (x);                                                            \
        if (_r != ncclSuccess) return fail(HAKAI_ERR_COMM, "%s: %s", #x, ncclGetErrorString(_r)); \
    } while (0)

namespace {

__global__ void k_save_upre(const int* up, int n_up, const int* dn, int n_dn, const double* upre, double* saved) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_up + n_dn) return;
    const long long n = j < n_up ? up[j] : dn[j - n_up];
    saved[3 * j + 0] = upre[3 * n + 0];
    saved[3 * j + 1] = upre[3 * n + 1];
    saved[3 * j + 2] = upre[3 * n + 2];
}

__global__ void k_pack(const int* up, int n_up, const int* dn, int n_dn, const int* ptr, const int* inc,
                       const double* fe, int nslot, double* up_sendP, double* dn_sendC) {
#pragma clang fp contract(off)
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n_up) {
        const int n = up[j];
        double q0 = 0.0, q1 = 0.0, q2 = 0.0;
        for (int i = ptr[n]; i < ptr[n + 1]; ++i) {
            const double* f = fe + inc[i];
            q0 += f[0];
            q1 += f[1];
            q2 += f[2];
        }
        up_sendP[3 * j + 0] = q0;
        up_sendP[3 * j + 1] = q1;
        up_sendP[3 * j + 2] = q2;
    } else if (j < n_up + n_dn) {
        const int jj = j - n_up;
        const int n = dn[jj];
        const int b = ptr[n], m = ptr[n + 1] - b;
        double* o = dn_sendC + (long long)3 * nslot * jj;
        for (int s = 0; s < nslot; ++s) {
            if (s < m) {
                const double* f = fe + inc[b + s];
                o[3 * s + 0] = f[0];
                o[3 * s + 1] = f[1];
                o[3 * s + 2] = f[2];
            } else {
                o[3 * s + 0] = 0.0;
                o[3 * s + 1] = 0.0;
                o[3 * s + 2] = 0.0;
            }
        }
    }
}

// Re-does the central-difference update (v2/HAKAI_j.jl:564, same expression as k_nodal) for the
// interface nodes with the cross-rank Q.
__global__ void k_fix(const int* up, int n_up, const int* dn, int n_dn, const int* ptr, const int* inc,
                      const double* fe, int nslot, const double* up_sendP, const double* up_recvC,
                      const double* dn_recvP, const double* saved, const double* u, double* out, const double* mass,
                      const double* fext, double dt, const int* poison) {
#pragma clang fp contract(off)
    if (*poison) return;  // contact overflow earlier in the call: the state stays the last good step's
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_up + n_dn) return;
    double Q[3];
    long long n;
    if (j < n_up) {
        n = up[j];
        for (int c = 0; c < 3; ++c) Q[c] = up_sendP[3 * j + c];
        const double* r = up_recvC + (long long)3 * nslot * j;
        for (int s = 0; s < nslot; ++s)
            for (int c = 0; c < 3; ++c) Q[c] += r[3 * s + c];
    } else {
        const int jj = j - n_up;
        n = dn[jj];
        for (int c = 0; c < 3; ++c) Q[c] = dn_recvP[3 * jj + c];
        const int b = ptr[n], m = ptr[n + 1] - b;
        for (int s = 0; s < nslot; ++s) {
            if (s < m) {
                const double* f = fe + inc[b + s];
                for (int c = 0; c < 3; ++c) Q[c] += f[c];
            } else {
                for (int c = 0; c < 3; ++c) Q[c] += 0.0;
            }
        }
    }
    const double m_ = mass[n];
    const double dC = 0.0 * m_;
    const double mdt2 = m_ / (dt * dt);
    const double inv = 1.0 / (mdt2 + dC / 2.0 / dt);
    for (int c = 0; c < 3; ++c) {
        const double uc = u[3 * n + c];
        const double up_ = saved[3 * j + c];
        const double f = fext ? fext[3 * n + c] : 0.0;  // contact force (external_force, :500-564)
        out[3 * n + c] = inv * (f - Q[c] + mdt2 * (2.0 * uc - up_) + dC / 2.0 / dt * up_);
    }
}

// Owner-computed assembly (hakai_capi.cpp own_build): a node's local Q is own_q[n] plus its rows
// (own_ridx[own_rp[n]..]) in element order, and every local contribution of a dn node is a row of
// its own -- so the partial sums and single contributions below are those k_pack / k_fix take
// from fe, in the same order.
__global__ void k_pack_own(const int* up, int n_up, const int* dn, int n_dn, const int* rp, const int* ridx,
                           const double* rows, const double* own_q, int nslot, double* up_sendP, double* dn_sendC) {
#pragma clang fp contract(off)
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n_up) {
        const int n = up[j];
        double q[3] = {own_q[3LL * n], own_q[3LL * n + 1], own_q[3LL * n + 2]};
        for (int i = rp[n]; i < rp[n + 1]; ++i)
            for (int c = 0; c < 3; ++c) q[c] += rows[3LL * ridx[i] + c];
        for (int c = 0; c < 3; ++c) up_sendP[3 * j + c] = q[c];
    } else if (j < n_up + n_dn) {
        const int jj = j - n_up;
        const int n = dn[jj];
        const int b = rp[n], m = rp[n + 1] - b;
        double* o = dn_sendC + (long long)3 * nslot * jj;
        for (int s = 0; s < nslot; ++s)
            for (int c = 0; c < 3; ++c) o[3 * s + c] = s < m ? rows[3LL * ridx[b + s] + c] : 0.0;
    }
}

__global__ void k_fix_own(const int* up, int n_up, const int* dn, int n_dn, const int* rp, const int* ridx,
                          const double* rows, int nslot, const double* up_sendP, const double* up_recvC,
                          const double* dn_recvP, const double* saved, const double* u, double* out, const double* mass,
                          const double* fext, double dt, const int* poison) {
#pragma clang fp contract(off)
    if (*poison) return;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_up + n_dn) return;
    double Q[3];
    long long n;
    if (j < n_up) {
        n = up[j];
        for (int c = 0; c < 3; ++c) Q[c] = up_sendP[3 * j + c];
        const double* r = up_recvC + (long long)3 * nslot * j;
        for (int s = 0; s < nslot; ++s)
            for (int c = 0; c < 3; ++c) Q[c] += r[3 * s + c];
    } else {
        const int jj = j - n_up;
        n = dn[jj];
        for (int c = 0; c < 3; ++c) Q[c] = dn_recvP[3 * jj + c];
        const int b = rp[n], m = rp[n + 1] - b;
        for (int s = 0; s < nslot; ++s)
            for (int c = 0; c < 3; ++c) Q[c] += s < m ? rows[3LL * ridx[b + s] + c] : 0.0;
    }
    const double m_ = mass[n];
    const double dC = 0.0 * m_;
    const double mdt2 = m_ / (dt * dt);
    const double inv = 1.0 / (mdt2 + dC / 2.0 / dt);
    for (int c = 0; c < 3; ++c) {
        const double uc = u[3 * n + c];
        const double up_ = saved[3 * j + c];
        const double f = fext ? fext[3 * n + c] : 0.0;
        out[3 * n + c] = inv * (f - Q[c] + mdt2 * (2.0 * uc - up_) + dC / 2.0 / dt * up_);
    }
}

template <class T>
hipError_t dalloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    return hipMalloc((void**)p, n * sizeof(T));
}
template <class T>
void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

void free_iface(hkc::Comm* m) {
    dfree(m->d_up);
    dfree(m->d_dn);
    for (int p = 0; p < 2; ++p) {
        dfree(m->d_up_sendP[p]);
        dfree(m->d_dn_sendC[p]);
    }
    dfree(m->d_up_recvC);
    dfree(m->d_dn_recvP);
    dfree(m->d_saved);
    m->n_up = m->n_dn = 0;
    m->pending = false;
}

hkc::Comm* peer(hkc::Comm* m, int r) {
    if (!m->group || r < 0 || r >= m->nranks) return nullptr;
    hakai_ctx* c = m->group->ctx[r];
    return c ? c->comm : nullptr;
}

int comm_common_init(hakai_ctx* c, hkc::Comm* m) {
    if (hipStreamCreateWithFlags(&m->cs, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_packed[0], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_packed[1], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_ag_ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_ag_done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&m->ev_done, hipEventDisableTiming) != hipSuccess) {
        c->comm = m;
        hkc::comm_destroy(c);
        return fail(HAKAI_ERR_DEVICE, "comm_init: stream/event creation failed");
    }
    c->comm = m;
    return 0;
}

// In-process group all-gather: dst + off[q] <- src[q] (bytes[q]) for every rank q in ONE launch
// (the peers' buffers live on the same device; one kernel instead of a copy per rank). 8-byte
// words, then the tail bytes.
__global__ void k_gather_local(hkc::LocalGather g, char* dst) {
    const int q = (int)blockIdx.y;
    const char* src = g.src[q];
    char* out = dst + g.off[q];
    const long long nb = g.bytes[q];
    if (!src || nb <= 0) return;
    const long long nw = nb >> 3;
    const long long stride = (long long)gridDim.x * blockDim.x;
    const long long i0 = blockIdx.x * (long long)blockDim.x + threadIdx.x;
    for (long long i = i0; i < nw; i += stride)
        reinterpret_cast<unsigned long long*>(out)[i] = reinterpret_cast<const unsigned long long*>(src)[i];
    for (long long i = (nw << 3) + i0; i < nb; i += stride) out[i] = src[i];
}

}  // namespace

namespace hkc {

int gather_local(hakai_ctx* c, const LocalGather& g, int n, void* dst) {
    long long mx = 0;
    for (int q = 0; q < n; ++q) {
        if (((uintptr_t)g.src[q] | (uintptr_t)g.off[q]) & 7)
            return fail(HAKAI_ERR_ARG, "gather_local: rank %d block not 8-byte aligned", q);
        mx = std::max(mx, g.bytes[q]);
    }
    if (mx <= 0) return 0;
    const unsigned gx = (unsigned)std::min<long long>(std::max<long long>(((mx >> 3) + 255) / 256, 1), 512);
    hipLaunchKernelGGL(k_gather_local, dim3(gx, (unsigned)n), dim3(256), 0, c->stream, g, (char*)dst);
    HIPCHK(hipGetLastError());
    return 0;
}

void comm_destroy(hakai_ctx* c) {
    Comm* m = c->comm;
    if (!m) return;
    if (m->cs) (void)hipStreamSynchronize(m->cs);
    (void)hipStreamSynchronize(c->stream);
    free_iface(m);
    if (m->nc) (void)ncclCommDestroy(m->nc);
    if (m->group) {
        std::lock_guard<std::mutex> lk(g_groups_mu);
        m->group->ctx[m->rank] = nullptr;
        if (--m->group->refs == 0) {
            g_groups.erase(m->group_key);
            delete m->group;
        }
    }
    for (int p = 0; p < 2; ++p)
        if (m->ev_packed[p]) (void)hipEventDestroy(m->ev_packed[p]);
    if (m->ev_ag_ready) (void)hipEventDestroy(m->ev_ag_ready);
    if (m->ev_ag_done) (void)hipEventDestroy(m->ev_ag_done);
    if (m->ev_done) (void)hipEventDestroy(m->ev_done);
    if (m->cs) (void)hipStreamDestroy(m->cs);
    delete m;
    c->comm = nullptr;
}

bool comm_is_local(const hakai_ctx* c) {
    return c->comm && c->comm->mode == 1 && (c->comm->n_up + c->comm->n_dn > 0 || c->contact);
}

int comm_rank(const hakai_ctx* c) { return c->comm ? c->comm->rank : 0; }
int comm_size(const hakai_ctx* c) { return c->comm ? c->comm->nranks : 1; }

// RCCL only: recv[q*bytes .. (q+1)*bytes) = rank q's `send`, ordered on c->stream (the divided
// contact search's per-step event exchange, hakai_contact.hip)
int comm_allgather_raw(hakai_ctx* c, const void* send, void* recv, size_t bytes) {
    Comm* m = c->comm;
    if (!m || m->mode != 0) return fail(HAKAI_ERR_STATE, "all-gather: not an RCCL communicator");
    if (bytes == 0) return 0;
    HIPCHK(hipEventRecord(m->ev_ag_ready, c->stream));
    HIPCHK(hipStreamWaitEvent(m->cs, m->ev_ag_ready, 0));
    NCCLCHK(ncclAllGather(send, recv, bytes, ncclUint8, m->nc, m->cs));
    HIPCHK(hipEventRecord(m->ev_ag_done, m->cs));
    HIPCHK(hipStreamWaitEvent(c->stream, m->ev_ag_done, 0));
    return 0;
}

// RCCL only: every rank's block, each at its own size (bytes[q]), into recv + off[q] for q != this
// rank (this rank's block stays in `send`); one grouped ncclSend/ncclRecv per peer, ordered on
// c->stream. The multi-GPU contact's exchanges: each block is sized by what its rank produced, so
// a rank with few records sends few bytes (an all-gather moves nranks x the largest block).
int comm_allgatherv_raw(hakai_ctx* c, const void* send, void* recv, const size_t* bytes, const size_t* off) {
    Comm* m = c->comm;
    if (!m || m->mode != 0) return fail(HAKAI_ERR_STATE, "all-gather: not an RCCL communicator");
    HIPCHK(hipEventRecord(m->ev_ag_ready, c->stream));
    HIPCHK(hipStreamWaitEvent(m->cs, m->ev_ag_ready, 0));
    NCCLCHK(ncclGroupStart());
    for (int q = 0; q < m->nranks; ++q) {
        if (q == m->rank) continue;
        if (bytes[m->rank]) NCCLCHK(ncclSend(send, bytes[m->rank], ncclUint8, q, m->nc, m->cs));
        if (bytes[q]) NCCLCHK(ncclRecv(static_cast<char*>(recv) + off[q], bytes[q], ncclUint8, q, m->nc, m->cs));
    }
    NCCLCHK(ncclGroupEnd());
    HIPCHK(hipEventRecord(m->ev_ag_done, m->cs));
    HIPCHK(hipStreamWaitEvent(c->stream, m->ev_ag_done, 0));
    return 0;
}

// RCCL only: recv = elementwise MIN over the ranks of send (uint64 words), ordered on c->stream
// (the multi-GPU contact's pair boxes, hakai_contact.hip)
int comm_allreduce_min_u64(hakai_ctx* c, const void* send, void* recv, size_t count) {
    Comm* m = c->comm;
    if (!m || m->mode != 0) return fail(HAKAI_ERR_STATE, "all-reduce: not an RCCL communicator");
    if (count == 0) return 0;
    HIPCHK(hipEventRecord(m->ev_ag_ready, c->stream));
    HIPCHK(hipStreamWaitEvent(m->cs, m->ev_ag_ready, 0));
    NCCLCHK(ncclAllReduce(send, recv, count, ncclUint64, ncclMin, m->nc, m->cs));
    HIPCHK(hipEventRecord(m->ev_ag_done, m->cs));
    HIPCHK(hipStreamWaitEvent(c->stream, m->ev_ag_done, 0));
    return 0;
}

bool comm_is_rccl(const hakai_ctx* c) { return c->comm && c->comm->mode == 0; }

// in-process group: the context of rank q (null otherwise)
hakai_ctx* comm_peer_ctx(hakai_ctx* c, int q) {
    Comm* m = c->comm;
    if (!m || m->mode != 1 || !m->group || q < 0 || q >= m->nranks) return nullptr;
    return m->group->ctx[q];
}

int comm_reset(hakai_ctx* c) {
    if (c->comm) c->comm->pending = false;
    return 0;
}

// the interface exchange the next nodal update consumes: (pending, buffer parity)
void comm_pending_get(const hakai_ctx* c, bool* pending, int* par) {
    *pending = c->comm && c->comm->pending;
    *par = c->comm ? c->comm->pending_par : 0;
}

// A poisoned call was rolled back to the state after step `last_good` (finish_call). Its
// state-writing kernels were no-ops from the poisoned step on, but every step still packed its
// interface forces -- from the unchanged sums of the last good step -- into the parity of its own
// step number. The next nodal update must read the parity of the last good step, not the last
// packed one: the step run again packs into the other parity, and an in-process peer that pulls
// after it (hakai_step_group runs the ranks one after another) would otherwise read the new sums.
// had_good: some step of the call ran; otherwise (pending, par) are the call's starting values.
void comm_rollback(hakai_ctx* c, bool had_good, long long last_good, bool pending, int par) {
    Comm* m = c->comm;
    if (!m) return;
    if (had_good) {
        m->pending = m->n_up + m->n_dn > 0;
        m->pending_par = (int)(last_good & 1);
    } else {
        m->pending = pending;
        m->pending_par = par;
    }
}

const std::vector<int>* comm_dn_nodes(const hakai_ctx* c) { return c->comm ? &c->comm->h_dn : nullptr; }

int comm_pre_nodal(hakai_ctx* c) {
    Comm* m = c->comm;
    if (!m || m->n_up + m->n_dn == 0 || !m->pending) return 0;
    const int n = m->n_up + m->n_dn;
    hipLaunchKernelGGL(k_save_upre, dim3((n + 255) / 256), dim3(256), 0, c->stream, m->d_up, m->n_up, m->d_dn, m->n_dn,
                       c->d_u[1 - c->cur], m->d_saved);
    HIPCHK(hipGetLastError());
    return 0;
}

int comm_post_nodal(hakai_ctx* c, double d_time) {
    Comm* m = c->comm;
    if (!m || m->n_up + m->n_dn == 0 || !m->pending) return 0;
    m->pending = false;
    const int par = m->pending_par;
    EventPair ep;
    prof_begin(c, HAKAI_K_EXCHANGE, &ep);
    if (m->mode == 0) {
        HIPCHK(hipStreamWaitEvent(c->stream, m->ev_done, 0));
    } else {  // pull the neighbours' packed buffers of the previous step
        if (m->n_up) {
            Comm* p = peer(m, m->rank + 1);
            if (!p) return fail(HAKAI_ERR_COMM, "local group: rank %d missing", m->rank + 1);
            HIPCHK(hipStreamWaitEvent(c->stream, p->ev_packed[par], 0));
            HIPCHK(hipMemcpyAsync(m->d_up_recvC, p->d_dn_sendC[par], sizeof(double) * 3 * m->nslot * m->n_up,
                                  hipMemcpyDeviceToDevice, c->stream));
        }
        if (m->n_dn) {
            Comm* p = peer(m, m->rank - 1);
            if (!p) return fail(HAKAI_ERR_COMM, "local group: rank %d missing", m->rank - 1);
            HIPCHK(hipStreamWaitEvent(c->stream, p->ev_packed[par], 0));
            HIPCHK(hipMemcpyAsync(m->d_dn_recvP, p->d_up_sendP[par], sizeof(double) * 3 * m->n_dn,
                                  hipMemcpyDeviceToDevice, c->stream));
        }
    }
    if (!c->q_from_buf && c->own_valid) {  // the previous element step summed node forces itself
        const int n = m->n_up + m->n_dn;
        hipLaunchKernelGGL(k_fix_own, dim3((n + 255) / 256), dim3(256), 0, c->stream, m->d_up, m->n_up, m->d_dn,
                           m->n_dn, c->d_own_rp, c->d_own_ridx, c->d_own_rows, m->nslot, m->d_up_sendP[par],
                           m->d_up_recvC, m->d_dn_recvP, m->d_saved, c->d_u[c->cur], c->d_u[1 - c->cur], c->d_mass,
                           c->contact ? c->d_fext : nullptr, d_time, c->d_poison);
        HIPCHK(hipGetLastError());
    } else if (!c->q_from_buf) {  // an uploaded Q already holds the global sum
        const int n = m->n_up + m->n_dn;
        hipLaunchKernelGGL(k_fix, dim3((n + 255) / 256), dim3(256), 0, c->stream, m->d_up, m->n_up, m->d_dn, m->n_dn,
                           c->d_inc_ptr, c->d_inc, c->d_fe, m->nslot, m->d_up_sendP[par], m->d_up_recvC, m->d_dn_recvP,
                           m->d_saved, c->d_u[c->cur], c->d_u[1 - c->cur], c->d_mass, c->contact ? c->d_fext : nullptr,
                           d_time, c->d_poison);
        HIPCHK(hipGetLastError());
    }
    prof_end(c, &ep);
    return 0;
}

int comm_post_element(hakai_ctx* c, long long step) {
    Comm* m = c->comm;
    if (!m || m->n_up + m->n_dn == 0) return 0;
    const int par = (int)(step & 1);
    const int n = m->n_up + m->n_dn;
    if (c->own_valid)  // this step's element kernel summed the node forces (owner-computed assembly)
        hipLaunchKernelGGL(k_pack_own, dim3((n + 255) / 256), dim3(256), 0, c->stream, m->d_up, m->n_up, m->d_dn,
                           m->n_dn, c->d_own_rp, c->d_own_ridx, c->d_own_rows, c->d_own_q, m->nslot,
                           m->d_up_sendP[par], m->d_dn_sendC[par]);
    else
        hipLaunchKernelGGL(k_pack, dim3((n + 255) / 256), dim3(256), 0, c->stream, m->d_up, m->n_up, m->d_dn, m->n_dn,
                           c->d_inc_ptr, c->d_inc, c->d_fe, m->nslot, m->d_up_sendP[par], m->d_dn_sendC[par]);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(m->ev_packed[par], c->stream));
    if (m->mode == 0) {
        HIPCHK(hipStreamWaitEvent(m->cs, m->ev_packed[par], 0));
        NCCLCHK(ncclGroupStart());
        if (m->n_up) {
            NCCLCHK(ncclSend(m->d_up_sendP[par], (size_t)3 * m->n_up, ncclDouble, m->rank + 1, m->nc, m->cs));
            NCCLCHK(ncclRecv(m->d_up_recvC, (size_t)3 * m->nslot * m->n_up, ncclDouble, m->rank + 1, m->nc, m->cs));
        }
        if (m->n_dn) {
            NCCLCHK(ncclSend(m->d_dn_sendC[par], (size_t)3 * m->nslot * m->n_dn, ncclDouble, m->rank - 1, m->nc, m->cs));
            NCCLCHK(ncclRecv(m->d_dn_recvP, (size_t)3 * m->n_dn, ncclDouble, m->rank - 1, m->nc, m->cs));
        }
        NCCLCHK(ncclGroupEnd());
        HIPCHK(hipEventRecord(m->ev_done, m->cs));
    }
    m->pending = true;
    m->pending_par = par;
    return 0;
}

}  // namespace hkc

extern "C" {

int hakai_comm_unique_id(uint8_t id[128]) {
    if (!id) return fail(HAKAI_ERR_ARG, "null id");
    static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
    ncclUniqueId u;
    NCCLCHK(ncclGetUniqueId(&u));
    std::memcpy(id, &u, 128);
    return 0;
}

int hakai_comm_init(hakai_ctx* c, int rank, int nranks, const uint8_t id[128]) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(HAKAI_ERR_ARG, "comm_init: bad args");
    HIPCHK(hipSetDevice(c->device));
    hkc::comm_destroy(c);
    hkc::Comm* m = new hkc::Comm();
    m->rank = rank;
    m->nranks = nranks;
    ncclUniqueId u;
    std::memcpy(&u, id, 128);
    ncclResult_t r = ncclCommInitRank(&m->nc, nranks, u, rank);
    if (r != ncclSuccess) {
        delete m;
        return fail(HAKAI_ERR_COMM, "ncclCommInitRank: %s", ncclGetErrorString(r));
    }
    return comm_common_init(c, m);
}

int hakai_comm_init_local(hakai_ctx* c, int rank, int nranks, int64_t group_key) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c || nranks < 1 || rank < 0 || rank >= nranks) return fail(HAKAI_ERR_ARG, "comm_init_local: bad args");
    HIPCHK(hipSetDevice(c->device));
    hkc::comm_destroy(c);
    hkc::Comm* m = new hkc::Comm();
    m->mode = 1;
    m->rank = rank;
    m->nranks = nranks;
    m->group_key = group_key;
    {
        std::lock_guard<std::mutex> lk(hkc::g_groups_mu);
        hkc::LocalGroup*& g = hkc::g_groups[group_key];
        if (!g) {
            g = new hkc::LocalGroup();
            g->nranks = nranks;
            g->ctx.assign(nranks, nullptr);
        }
        if (g->nranks != nranks || g->ctx[rank]) {
            delete m;
            return fail(HAKAI_ERR_ARG, "comm_init_local: group %lld size/rank clash", (long long)group_key);
        }
        // the group's kernels read the peers' buffers directly (k_gather_local, the phase-B event
        // gather) and no peer access is enabled: every member must live on one device
        for (int q = 0; q < nranks; ++q)
            if (g->ctx[q] && g->ctx[q]->device != c->device) {
                delete m;
                return fail(HAKAI_ERR_ARG, "comm_init_local: rank %d is on device %d but rank %d of group %lld is on "
                            "device %d; an in-process group shares one device (use hakai_comm_init, RCCL, across "
                            "devices)", rank, c->device, q, (long long)group_key, g->ctx[q]->device);
            }
        g->ctx[rank] = c;
        g->refs++;
        m->group = g;
    }
    return comm_common_init(c, m);
}

int hakai_set_interface(hakai_ctx* c, int64_t n_shared, const int64_t* local_node, const int32_t* rank_lo,
                        const int32_t* rank_hi) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    hkc::Comm* m = c->comm;
    if (!m) return fail(HAKAI_ERR_STATE, "set_interface before comm_init");
    if (!c->model_ok) return fail(HAKAI_ERR_STATE, "set_interface before upload_model");
    if (n_shared < 0 || (n_shared > 0 && (!local_node || !rank_lo || !rank_hi)))
        return fail(HAKAI_ERR_ARG, "set_interface: bad arrays");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipStreamSynchronize(m->cs));
    free_iface(m);
    std::vector<int> up, dn;
    for (int64_t j = 0; j < n_shared; ++j) {
        if (rank_hi[j] != rank_lo[j] + 1)
            return fail(HAKAI_ERR_ARG, "set_interface: node shared by ranks %d..%d; only adjacent-rank sharing is supported",
                        rank_lo[j], rank_hi[j]);
        if (local_node[j] < 0 || local_node[j] >= c->nN) return fail(HAKAI_ERR_ARG, "set_interface: node out of range");
        if (rank_lo[j] == m->rank) up.push_back((int)local_node[j]);
        else if (rank_hi[j] == m->rank) dn.push_back((int)local_node[j]);
        else return fail(HAKAI_ERR_ARG, "set_interface: node %lld not shared with this rank", (long long)local_node[j]);
    }
    if ((!up.empty() && m->rank + 1 >= m->nranks) || (!dn.empty() && m->rank == 0))
        return fail(HAKAI_ERR_ARG, "set_interface: neighbour rank does not exist");
    // Slots = max incidences the upper side holds at a shared node. For RCCL all ranks agree via an
    // all-reduce; a local group uses the structural bound 8 (hex8: <= 8 incidences per node on
    // structured meshes, padded with zeros, which leaves the sums unchanged).
    std::vector<int> ptr((size_t)c->nN + 1);
    HIPCHK(hipMemcpy(ptr.data(), c->d_inc_ptr, ptr.size() * sizeof(int), hipMemcpyDeviceToHost));
    int nslot = 0;
    for (int n : dn) nslot = std::max(nslot, ptr[n + 1] - ptr[n]);
    if (m->mode == 0) {
        int* d_ns = nullptr;
        HIPCHK(dalloc(&d_ns, 1));
        HIPCHK(hipMemcpy(d_ns, &nslot, sizeof(int), hipMemcpyHostToDevice));
        NCCLCHK(ncclAllReduce(d_ns, d_ns, 1, ncclInt32, ncclMax, m->nc, m->cs));
        HIPCHK(hipStreamSynchronize(m->cs));
        HIPCHK(hipMemcpy(&nslot, d_ns, sizeof(int), hipMemcpyDeviceToHost));
        dfree(d_ns);
    } else {
        if (nslot > 8) return fail(HAKAI_ERR_ARG, "local group: node with %d incidences on the upper side", nslot);
        nslot = 8;
    }
    m->nslot = nslot;
    m->n_up = (int)up.size();
    m->n_dn = (int)dn.size();
    m->h_dn = dn;
    c->own_built_g = -1;  // owner-assembly lists export every dn node's contributions: rebuilt
    c->own_for_g0 = -1;
    c->own_valid = false;
    HIPCHK(dalloc(&m->d_up, up.size()));
    HIPCHK(dalloc(&m->d_dn, dn.size()));
    for (int p = 0; p < 2; ++p) {
        HIPCHK(dalloc(&m->d_up_sendP[p], 3 * up.size()));
        HIPCHK(dalloc(&m->d_dn_sendC[p], 3 * (size_t)nslot * dn.size()));
    }
    HIPCHK(dalloc(&m->d_up_recvC, 3 * (size_t)nslot * up.size()));
    HIPCHK(dalloc(&m->d_dn_recvP, 3 * dn.size()));
    HIPCHK(dalloc(&m->d_saved, 3 * (up.size() + dn.size())));
    if (!up.empty()) HIPCHK(hipMemcpy(m->d_up, up.data(), up.size() * sizeof(int), hipMemcpyHostToDevice));
    if (!dn.empty()) HIPCHK(hipMemcpy(m->d_dn, dn.data(), dn.size() * sizeof(int), hipMemcpyHostToDevice));
    m->pending = false;
    return 0;
}

}  // extern "C"
