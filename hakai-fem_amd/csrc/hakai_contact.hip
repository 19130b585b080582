// hakai_contact.hip -- all-exterior instance-vs-instance contact on gfx950.
//
// Reference: v2/HAKAI_j.jl (v2 = HAKAI-v0.0.2/Julia)
//   setup            :244-421   pairs (instance_pair, cp_index), CT lists, element sizes
//   get_element_face :1944-1992, get_surface_triangle :1996-2164, add_surface_triangle :2167-2245
//   surface update   :766-804   (after element deletion)
//   cal_contact_force:2248-2706 (CPU path; the CUDA.jl path :2899-3157 deliberately differs, §9 Q14)
//   accumulation     :435, :511-538  (Float128 per thread, rounded once into external_force)
//
// Design (MI355X-first, same results):
//   * The contact lists the reference grows at run time (appending newly exposed faces when an
//     element is deleted) are enumerated ONCE on the host: every triangle / contact node that can
//     ever appear carries the elements whose deletion adds it. On the device an entry is live at
//     step t iff it was in the initial list or one of its adders was deleted before t (del_step).
//     Same sets as the reference at every step, no host round trip, no reallocation.
//   * The reference's candidate filter |cell(j0) - cell(i)| <= 1 per axis (cells of size
//     1.1*elementMaxSize, 0.6 for self-contact) becomes a hash grid over the i-nodes: a triangle
//     visits the distinct buckets of the 27 neighbouring cells and applies the exact same integer
//     test, so the candidate set is identical and the work is O(contact nodes), not O(T x N).
//   * Every contact event computes the reference's FP64 expressions verbatim (no contraction).
//     Forces are gathered per node and summed in double-double, then rounded once: the reference
//     sums in Float128 and rounds once, so both are the correctly rounded sum up to a 2^-106
//     relative window (order-independent, no atomics on doubles).
#include <hip/hip_runtime.h>


#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <vector>

#include "hakai_internal.hpp"

using hkc::fail;
using hkc::hip_fail;

#define HIPCHK(x)                                      \
    do {                                               \
        hipError_t _e = (x);                           \
        if (_e != hipSuccess) return hip_fail(_e, #x); \
    } while (0)

namespace hkc {

struct PairParam {
    double young, kc, Cr, ddiv;
    int self;
    int hash_off, hash_size;
    int pad;
};

// Multi-GPU contact (hakai_set_contact_global, §8f-3): owner-computed search. Every rank sets up
// the contact model of the GLOBAL mesh (the same host enumeration, so the same entries, pairs and
// hash tables on every rank) and keeps the entries it owns: the triangles of its own elements and
// the node entries of the nodes it owns (owner = the rank of the node's lowest incident element),
// with local node ids, so every position, velocity and element flag the search reads is local. Per
// step (hkc::Xrank, "exchange" kernels below):
//   A1  the previous step's deletions of every rank (global element, step) are all-gathered into a
//       global deletion-step array (live lists: an entry's adders may sit on a neighbour rank);
//       live-list update of the own entries; pair boxes over the own live node entries;
//   A2  the partial boxes are combined (an all-reduce of min/max words, exact); the own live
//       i-nodes inside the pair's range box are binned into compact 96-B records (cell, global
//       node, position, velocity, the mass the damping term reads);
//   A3  the records of every rank are gathered into one hash grid (count, scan, fill), and each
//       rank tests its own candidate triangles (the reference's triangle-parallel loop :2370,
//       per-thread force columns :2386) against every binned i-node: the same candidate set and the
//       same FP64 expressions as one GPU;
//   B   the events of all ranks are all-gathered and every rank forms the same order-independent
//       double-double sums (:2653-2667, :511-517), then takes its own nodes' forces.
// So N ranks are bit-identical to one, and nothing of the model's surface travels per step: only
// deletions, the boxes, the binned contact-zone nodes and the events. Blocks are double-buffered by
// step parity; an in-process group reads its peers' blocks directly (after a stream wait on their
// "packed" events), RCCL all-gathers them. Block capacities (RCCL collectives need host-known
// sizes) are the same on every rank and grow between steps from the counts every rank gathered
// two steps earlier; a burst beyond a capacity poisons that step on every rank, and hakai_step
// grows the capacity and runs the step again (contact_exchange_retry).
// Exchange blocks of every rank: rank q's block at p[q] (RCCL receive buffer or in-process peer)
constexpr int kMaxXRanks = 64;
struct XBlk {
    const char* p[kMaxXRanks];
    int cap[kMaxXRanks];  // records rank q's block holds
    int off[kMaxXRanks];  // prefix of cap: rank q's first slot in arrays over every rank's records
};

struct Xrank {
    int rank = 0, nranks = 1;
    long long E0 = 0, nEloc = 0, nN_g = 0, nE_g = 0;
    int maxEloc = 1;                  // the largest rank's element count (full deletion blocks)
    long long* d_eoff = nullptr;      // [nranks+1] element ranges
    int* d_l2g = nullptr;             // [nN local] global node id
    int* d_g2l = nullptr;             // [nN_g] local node id or -1
    double* g_mass = nullptr;         // [nN_g] lumped node mass (diag_M[i] with a node id i, :2592)
    int* g_del = nullptr;             // [nE_g + 2] deletion step; [nE_g + 1] last step with any deletion
    int* d_last_del = nullptr;        // [nEloc] local deletion steps at the last pack
    // exchange blocks: int4 header (count, overflow, last deletion step, full) + records
    static constexpr int kNx = 3;     // 0 deletions, 1 binned i-nodes, 2 events
    char* d_send[kNx][2] = {{nullptr, nullptr}, {nullptr, nullptr}, {nullptr, nullptr}};
    size_t send_bytes[kNx] = {0, 0, 0};
    char* d_recv[kNx] = {nullptr, nullptr, nullptr};   // RCCL: [nranks] blocks
    size_t recv_bytes[kNx] = {0, 0, 0};
    // records per block: capq[x][q] for rank q's block, computed alike on every rank from the
    // gathered counts (so every rank knows every block's size); cap[x] = their maximum
    long long cap[kNx] = {0, 0, 0};
    std::vector<long long> capq[kNx];
    std::vector<int> hist[kNx];       // [q][kHist] recent gathered counts of each rank (the headroom window)
    int hist_pos = 0;
    static constexpr int kHist = 16;
    long long cap_max[kNx] = {0, 0, 0};
    long long cap_floor[kNx] = {1024, 256, 256};  // smallest capacity (tuning contact_exchange_*)
    hipEvent_t ev_sent[kNx][2] = {{nullptr, nullptr}, {nullptr, nullptr}, {nullptr, nullptr}};
    bool full_del = true;             // the next deletion block carries every local deletion step
    // partial pair boxes of this rank, by parity (in-process peers read them), and the combined boxes
    unsigned long long* d_box[2] = {nullptr, nullptr};
    unsigned long long* d_boxg = nullptr;
    hipEvent_t ev_box[2] = {nullptr, nullptr};
    int* d_xctl = nullptr;            // [0] exchange overflow bits of the current call (1 del, 2 bins, 4 events);
                                      // [4 ..] the step's gathered counts [kNx][nranks], then their
                                      // maxima since the last overflow growth [kNx][nranks]
    bool retry = false;               // the last poisoned call overflowed an exchange, now grown
    int* h_cnt = nullptr;             // pinned, device-mapped [4][kNx][nranks] gathered counts, written by
    int* d_hcnt = nullptr;            // the kernels that read the blocks (d_hcnt: device view), read two steps later
    hipEvent_t ev_cnt[4] = {nullptr, nullptr, nullptr, nullptr};
    long long seq = 0;                // steps since the last state reset: block parity, count ring
    long long cnt_seq = 0;            // count-ring entries written
    int sl_a = 0;                     // count-ring slot of the current step
    int t_a = 0;                      // step of the current phase A
    long long phase_a = 0;            // phase-A3 calls (equal on the ranks of a lockstep group)
    int par_a = 0;                    // parity of the blocks of the current step
};

// A hash-bucket entry: the i-node's cell, node id and position (coord + u of this step, the value
// the triangle test would gather: the same expression, so the same bits), written by the binning
// straight into the bucket list, so the triangle search reads one 64-B record per entry and has no
// dependent gather of the node's position behind it. next: the bucket's next entry (-1 = end).
struct alignas(16) BEnt {
    long long m[3];
    int node, pad;
    double p[3];
    long long next;
};
static_assert(sizeof(BEnt) == 64, "BEnt: four 16-B vectors");

// What an event's force needs from its i-node besides the position: the velocity (d_disp / d_time
// of the previous step, :628, or the initial velocity) and the mass the damping term reads
// (diag_M[i] with the node id i, :2592). Formed by the binning (same expressions, same bits) and
// kept beside the bucket list, so the search loads it only for an event.
struct alignas(16) BVel {
    double v[3], mq;
};
// A binned i-node as it travels between ranks (multi-GPU, A2 -> A3); pad of BEnt = the pair.
struct alignas(16) BRec {
    BEnt e;
    BVel w;
};
static_assert(sizeof(BRec) == 96, "BRec: six 16-B vectors");

struct Contact {
    // node / element space of the kernels: the context's own (one GPU) or the global mirror
    long long nN = 0, nE = 0;
    Xrank* xr = nullptr;             // multi-GPU (hakai_set_contact_global), else null
    int npairs = 0;
    std::vector<PairParam> h_par;
    PairParam* d_par = nullptr;
    // i-side (contact points) and j-side (triangle nodes) node entries, all pairs concatenated
    int n_ni = 0, n_nj = 0;
    int *d_ni_pair = nullptr, *d_ni_node = nullptr, *d_ni_orig = nullptr, *d_ni_aptr = nullptr, *d_ni_add = nullptr;
    int *d_nj_pair = nullptr, *d_nj_node = nullptr, *d_nj_orig = nullptr, *d_nj_aptr = nullptr, *d_nj_add = nullptr;
    int nseg = 0;
    int* d_seg = nullptr;  // [nseg] Seg: node-entry segment (start, end, pair, side, region)
    // triangles
    int n_tri = 0;
    int *d_tri_pair = nullptr, *d_tri_nodes = nullptr, *d_tri_ele = nullptr, *d_tri_adder = nullptr;
    // live lists (rebuilt on steps where the surface may have changed)
    int ntile = 0, nreg = 0;
    void* d_tiles = nullptr;        // [ntile] Tile
    int *d_tile_cnt = nullptr, *d_tile_off = nullptr;            // [ntile], [ntile+1]
    int* d_reg_first = nullptr;     // [nreg+1] first tile of each region
    int* d_reg = nullptr;           // [nreg][2] (base, live count)
    int* d_pair_reg = nullptr;      // [npairs][2] region of (pair, side)
    int tri_reg = 0;
    std::vector<int> reg_list_h;    // [nreg] list of each region (0 i-nodes, 1 j-nodes, 2 triangles)
    // element -> entries its deletion exposes (CSR), and the deleted-element list of a step
    int *d_el_tri_ptr = nullptr, *d_el_tri = nullptr, *d_el_ni_ptr = nullptr, *d_el_ni = nullptr;
    int *d_el_nj_ptr = nullptr, *d_el_nj = nullptr, *d_dlist = nullptr;
    int *d_ni_live = nullptr, *d_nj_live = nullptr, *d_tri_live = nullptr;
    bool force_rebuild = true;
    bool always_rebuild = false;    // tuning/testing: full rebuild every step (no incremental update)
    long long last_t = -1;
    // launch grids sized at setup from the contact model (small decks: few blocks, so the ~20
    // per-step kernels are not dominated by dispatching idle workgroups); every loop is grid-stride
    int g_seg = 256, g_ev = 1024, g_tri = 4096, g_node = 256, g_del = 1024, g_reset = 64;
    int g_box = 32;  // bounding boxes: blocks per segment (each block ends in 6 atomics on the pair's
                     // 6 bounds, so fewer, longer blocks: ~4 entries per thread, one unrolled pass)
    // hash grid over i-nodes
    int htot = 0;
    // bucket heads: (search sequence << 32 | first entry); a head of an older sequence is an empty
    // bucket, so the table is never cleared (chained buckets: no count, scan or fill pass)
    unsigned long long* d_head = nullptr;  // [htot]
    BEnt* d_blist = nullptr;        // [blist_cap] bucket lists
    BVel* d_bvel = nullptr;         // [blist_cap] beside them
    long long blist_cap = 0;
    unsigned long long* d_bbox = nullptr;  // [npairs][12] ordered-integer encoded doubles
    // small decks (set at setup; tuning "contact_fuse_small"): fused single-workgroup phases
    bool small = false;
    int fuse_small = 1;
    int fuse_binfilter = 1;  // tuning "contact_fuse_binfilter": binning and prefilter in one launch

    // events and per-node gather over the touched nodes
    long long cap = 0;
    unsigned int* d_ctl = nullptr;  // kCtl control words (events, max events, dirty, touched counts)
    unsigned int* d_evs = nullptr;  // [kEvShards][kShardStride] event counters (one per shard)
    int* d_ev_nodes = nullptr;      // [cap][4]
    double* d_ev_f = nullptr;       // [cap][3]
    int* d_cnt = nullptr;           // [nN] terms per node (zero between steps)
    int* d_tpos = nullptr;          // [nN] position of a touched node in its list
    int* d_touched[2] = {nullptr, nullptr};  // ping-pong lists of nodes with contact force
    int tsel = 0;
    long long tcap = 0;
    int* d_toff = nullptr;          // [tcap] start of each touched node's term range
    int* d_tcnt = nullptr;          // [tcap] its length
    void* d_cand = nullptr;         // [cand_cap] TriRec of the triangles passing the prefilter, in
                                    // kCandShards shards of cshard_cap records
    long long cand_cap = 0, cshard_cap = 0;
    unsigned int* d_ccnt = nullptr; // [kCandShards * kShardStride] candidate count of each shard (word
                                    // 0) and item count (word kItemWord)
    uint2* d_item = nullptr;        // [kCandShards][kItemsPerCand * cshard_cap] (candidate slot, cell << 27 |
                                    // bucket): the cells of a candidate's neighbourhood that its sphere reaches
    double* d_terms = nullptr;      // [4 cap][3]
    // velocity before the first step (initial condition / uploaded), v2/HAKAI_j.jl:233-239
    double* d_velo0 = nullptr;
    bool use_velo0 = true;
    double min_size = 0, max_size = 0, d_lim = 0;
    double myu = 0.25, kc_o = 1.0, kc_s = 1.0, Cr_o = 0.0, Cr_s = 0.0;  // :2255-2259
    std::vector<int> pair_inst;  // [npairs][2] (1-based instances), for hakai_contact_info
    std::vector<long long> pair_counts;  // [npairs][3] initial #nodes_i, #triangles, #nodes_j
};

}  // namespace hkc

namespace {

using hkc::Contact;
using hkc::PairParam;
using hkc::BEnt;
using hkc::BRec;
using hkc::BVel;

constexpr int kB = 256;

__device__ __forceinline__ unsigned long long enc(double d) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(d);
    return (u >> 63) ? ~u : (u | 0x8000000000000000ULL);
}
__device__ __forceinline__ double dec(unsigned long long e) {
    const unsigned long long u = (e >> 63) ? (e & 0x7FFFFFFFFFFFFFFFULL) : ~e;
    return __longlong_as_double((long long)u);
}

__device__ __forceinline__ bool live(int orig, const int* aptr, const int* add, int k, const int* del_step, int t) {
    if (orig) return true;
    for (int a = aptr[k]; a < aptr[k + 1]; ++a) {
        const int s = del_step[add[a]];  // -1: deleted before an upload_state
        if (s != 0 && s < t) return true;
    }
    return false;
}

__device__ __forceinline__ double my3norm(double a, double b, double c) {
#pragma clang fp contract(off)
    return sqrt(a * a + b * b + c * c);
}

__device__ __forceinline__ unsigned hash3(long long x, long long y, long long z) {
    const unsigned long long h = (unsigned long long)x * 0x9E3779B97F4A7C15ULL ^
                                 (unsigned long long)y * 0xC2B2AE3D27D4EB4FULL ^
                                 (unsigned long long)z * 0x165667B19E3779F9ULL;
    return (unsigned)(h ^ (h >> 29));
}

struct Range {
    double mn[3], mx[3], amn[3];
    bool empty;
};

__device__ __forceinline__ Range pair_range(const unsigned long long* bb_) {
    // the pair's 12 words as six 16-B loads, all in flight together (bbox + 12 * pair is 16-B aligned)
    unsigned long long bb[12];
#pragma unroll
    for (int w = 0; w < 6; ++w) {
        const ulonglong2 v = reinterpret_cast<const ulonglong2*>(bb_)[w];
        bb[2 * w] = v.x;
        bb[2 * w + 1] = v.y;
    }
    Range r;
    r.empty = false;
#pragma unroll
    for (int d = 0; d < 3; ++d) {  // branch-free: a side without live nodes makes the range empty
        const bool none = bb[d] == ~0ULL || bb[6 + d] == ~0ULL;
        const double mni = dec(bb[d]), mxi = dec(bb[3 + d]), mnj = dec(bb[6 + d]), mxj = dec(bb[9 + d]);
        r.empty |= none;
        r.mn[d] = none ? 0.0 : fmax(mni, mnj);
        r.mx[d] = none ? 0.0 : fmin(mxi, mxj);
        r.amn[d] = none ? 0.0 : fmin(mni, mnj);
    }
    if (!r.empty && (r.mn[0] > r.mx[0] || r.mn[1] > r.mx[1] || r.mn[2] > r.mx[2])) r.empty = true;  // :2304-2306
    return r;
}

// Control words (device): events this step, max events seen, full rebuild of the live lists,
// incremental update (an element was deleted in the previous step), deleted elements found, and
// the number of nodes with contact force in each of the two ping-pong "touched" lists.
enum { kEv = 0, kEvMax = 1, kDirty = 2, kDel = 3, kNdel = 4, kTouched = 5 /* [5], [6] */, kNcand = 7, kTerms = 8,
       kNcandMax = 9, kEvShardMax = 10, kCandShardMax = 11, kCandOver = 12, kSeq = 13, kItemShardMax = 14,
       kCtl = 16 };
// Events are appended into kEvShards shards, each with its own counter on its own 128-B line: with
// one counter, every wave that found an event waited on the same memory-side atomic (measured:
// 0.13 ms of a 0.30 ms contact step on C4).
constexpr int kEvShards = 64;
constexpr int kShardStride = 32;  // unsigned ints between shard counters
// Candidate triangles likewise: prefilter block b appends to shard b % kCandShards (one atomic per
// block on that shard's counter; clustered candidates fall in consecutive blocks, so shards stay even).
constexpr int kCandShards = 64;
constexpr int kItemWord = 1;       // a shard's item counter: with the candidate counter one 64-bit word
constexpr int kTestWord = 8;       // triangles the shard's prefilter blocks tested in full (stats)
constexpr int kItemsPerCand = 16;  // item capacity per candidate slot (a candidate has <= 27)
constexpr int kFilterBlocks = 2048;  // prefilter grid cap

// Step prologue: pair boxes to (+inf, -inf), event counter to 0, full rebuild if the host forces
// it, incremental update if an element was deleted in the previous step (del_any == t-1), and
// the contact forces of the previous step's touched nodes back to 0 (external_force is otherwise
// never rewritten).
// Counters the kernels of one launch read after other workgroups' (or, in the fused small-deck
// kernels, other waves') atomics: an agent-scope load, never a stale L1 line.
__device__ __forceinline__ unsigned ld_ctl(const unsigned int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The box array: 12 words per pair (pair_range), ordered-integer encoded doubles; min words start
// at +inf, max words at -inf (0).
__host__ __device__ __forceinline__ int box_words(int npairs) { return 12 * npairs; }
__device__ __forceinline__ bool box_max(int q) { return ((q % 12) / 3) % 2 == 1; }

// The per-step kernels below are bodies over (workgroup bid of nb): the __global__ wrappers pass
// blockIdx.x / gridDim.x, and the fused small-deck kernels (one workgroup, "Small decks") run
// several bodies back to back with a workgroup barrier between them.
// (multi-GPU: the touched nodes are global ids of this rank's nodes, g2l maps them into fext)
__device__ __forceinline__ void reset_body(int bid, int nb, unsigned long long* bbox, int npairs, unsigned int* ctl,
                                           unsigned int* evs, unsigned int* ccnt, int force, const int* del_any,
                                           int t, const double* t_rd, const int* touched_prev, int tsel,
                                           double* fext, const int* g2l = nullptr, int* zero_hdr = nullptr) {
    if (t_rd) t = (int)*t_rd + 1;  // graph mode: step number from the device counter
    const int i = bid * blockDim.x + threadIdx.x;
    if (zero_hdr && i < 2) zero_hdr[i] = 0;  // multi-GPU: this step's bin block (count, overflow)
    if (i < kEvShards) evs[i * kShardStride] = 0;
    if (i < kCandShards)
        ccnt[i * kShardStride] = ccnt[i * kShardStride + kTestWord] = ccnt[i * kShardStride + kItemWord] = 0;
    for (int q = i; q < box_words(npairs); q += nb * blockDim.x) bbox[q] = box_max(q) ? 0ULL : ~0ULL;
    if (i == 0) {
        ctl[kEv] = 0;
        ctl[kDirty] = force ? 1u : 0u;
        ctl[kDel] = (!force && del_any && *del_any == t - 1) ? 1u : 0u;
        ctl[kNdel] = 0;
        ctl[kNcand] = 0;
        ctl[kCandOver] = 0;
        ctl[kTerms] = 0;
        ctl[kTouched + tsel] = 0;
        ctl[kSeq] = ctl[kSeq] + 1u;  // this step's bucket-head stamp (never 0: the heads start at 0)
    }
    const int np = (int)ld_ctl(&ctl[kTouched + 1 - tsel]);
    for (int q = i; q < np; q += nb * blockDim.x) {
        const long long n = g2l ? g2l[touched_prev[q]] : touched_prev[q];  // (multi-GPU: only local nodes)
        fext[3 * n] = 0.0;
        fext[3 * n + 1] = 0.0;
        fext[3 * n + 2] = 0.0;
    }
}

__global__ void k_ct_reset(unsigned long long* bbox, int npairs, unsigned int* ctl, unsigned int* evs,
                           unsigned int* ccnt, int force, const int* del_any, int t, const double* t_rd,
                           const int* touched_prev, int tsel, double* fext, const int* g2l, int* zero_hdr) {
    reset_body(blockIdx.x, gridDim.x, bbox, npairs, ctl, evs, ccnt, force, del_any, t, t_rd, touched_prev, tsel,
               fext, g2l, zero_hdr);
}

struct StepIn {
    const double* coord;
    const double* u;       // disp at the start of the step
    const double* u_pre;   // disp_pre
    const double* velo0;   // non-null before the first step
    double d_time;
    const int* del_step;   // (multi-GPU: the global deletion steps)
    const int* flag;
    const int* conn;
    const double* mass;    // per node, indexed by global node id (multi-GPU: the global array)
    const int* l2g;        // multi-GPU: local -> global node id (null: the ids are global)
    int t;
};

__device__ __forceinline__ int gid(const StepIn& s, int n) { return s.l2g ? s.l2g[n] : n; }

// velocity of node n at the start of step t: the initial one before the first step, else d_disp /
// d_time of the previous step (:628)
__device__ __forceinline__ void velo(const StepIn& s, int n, double v[3]) {
#pragma clang fp contract(off)
    for (int c = 0; c < 3; ++c)
        v[c] = s.velo0 ? s.velo0[3 * n + c] : (s.u[3 * n + c] - s.u_pre[3 * n + c]) / s.d_time;
}

__device__ __forceinline__ void pos(const StepIn& s, int n, double p[3]) {
#pragma clang fp contract(off)
    for (int c = 0; c < 3; ++c) p[c] = s.coord[3 * n + c] + s.u[3 * n + c];  // position, :653-655
}

// ---- live lists -----------------------------------------------------------------------------
// Every node entry / triangle that can ever appear is enumerated at setup (most of them are
// interior and only become live if elements are deleted). The live ones are kept in index lists,
// one region per pair side's node segment (at the segment's own offset, capacity = segment size)
// and one for all triangles; reg[2r] = region base, reg[2r+1] = live count. Like the reference's
// c_nodes / c_triangles they only grow (:766-804): a deletion appends the entries it exposes
// (k_ct_append); triangles of deleted elements stay listed and are skipped at use (:2374-2377).
// A full rebuild (setup, state upload/reset, a probe, a non-consecutive step) scans everything
// in tiles of kTile entries that never straddle a region. Lists: 0 i-nodes, 1 j-nodes, 2 triangles.
constexpr int kTilePer = 8;
constexpr int kTile = kB * kTilePer;

struct LiveIn {
    const int *ni_orig, *ni_aptr, *ni_add, *nj_orig, *nj_aptr, *nj_add, *tri_ele, *tri_adder, *flag, *del_step;
    int t;
};

__device__ __forceinline__ bool is_live(const LiveIn& L, int list, int k) {
    if (list == 0) return live(L.ni_orig[k], L.ni_aptr, L.ni_add, k, L.del_step, L.t);
    if (list == 1) return live(L.nj_orig[k], L.nj_aptr, L.nj_add, k, L.del_step, L.t);
    const int ad = L.tri_adder[k];
    if (ad < 0) return true;
    const int st = L.del_step[ad];
    return st != 0 && st < L.t;  // face exposed by a deletion in an earlier step
}

// block-wide exclusive scan of one int per thread (blockDim.x <= 1024 threads, s_w[blockDim.x/64]);
// returns this thread's exclusive prefix, total = the block's sum
__device__ __forceinline__ int block_excl_scan(int v, int* s_w, int& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_w[w] = x;
    __syncthreads();
    int base = 0, tot = 0;
    const int nw = (int)blockDim.x >> 6;
    for (int q = 0; q < nw; ++q) {
        base += q < w ? s_w[q] : 0;
        tot += s_w[q];
    }
    __syncthreads();
    total = tot;
    return base + x - v;
}

struct Tile {
    int list, start, end, region;
};

__global__ __launch_bounds__(kB) void k_ct_live_count(const unsigned int* ctl, LiveIn L, const Tile* tiles,
                                                      int ntile, int* tile_cnt) {
    if (ctl[kDirty] == 0) return;
    __shared__ int s_w[kB / 64];
    for (int b = blockIdx.x; b < ntile; b += gridDim.x) {
        const Tile tl = tiles[b];
        int n = 0;
        for (int q = 0; q < kTilePer; ++q) {
            const int k = tl.start + (int)threadIdx.x + kB * q;
            if (k < tl.end && is_live(L, tl.list, k)) ++n;
        }
        int tot;
        block_excl_scan(n, s_w, tot);
        if (threadIdx.x == 0) tile_cnt[b] = tot;
    }
}

// one block: exclusive scan of the tile counts (tile_off[0..ntile]); region r = tiles
// [reg_first[r], reg_first[r+1]) -> reg[2r+1] = its live count
__global__ __launch_bounds__(kB) void k_ct_live_scan(const unsigned int* ctl, int ntile, const int* tile_cnt,
                                                     int* tile_off, int nreg, const int* reg_first, int* reg) {
    if (ctl[kDirty] == 0) return;
    __shared__ int s_w[kB / 64];
    int carry = 0;
    constexpr int PER = 16;
    for (int c0 = 0; c0 < ntile; c0 += kB * PER) {
        const int b = c0 + (int)threadIdx.x * PER;
        int v[PER], sum = 0;
        for (int q = 0; q < PER; ++q) {
            v[q] = b + q < ntile ? tile_cnt[b + q] : 0;
            sum += v[q];
        }
        int tot;
        int run = carry + block_excl_scan(sum, s_w, tot);
        for (int q = 0; q < PER; ++q) {
            if (b + q < ntile) tile_off[b + q] = run;
            run += v[q];
        }
        carry += tot;
    }
    if (threadIdx.x == 0) tile_off[ntile] = carry;
    __syncthreads();  // this block's global stores are visible to its own threads after the barrier
    for (int r = threadIdx.x; r < nreg; r += kB) reg[2 * r + 1] = tile_off[reg_first[r + 1]] - tile_off[reg_first[r]];
}

__global__ __launch_bounds__(kB) void k_ct_live_write(const unsigned int* ctl, LiveIn L, const Tile* tiles,
                                                      int ntile, const int* tile_off, const int* reg_first,
                                                      const int* reg, int* out_ni, int* out_nj, int* out_tri) {
    if (ctl[kDirty] == 0) return;
    __shared__ int s_w[kB / 64];
    for (int b = blockIdx.x; b < ntile; b += gridDim.x) {
        const Tile tl = tiles[b];
        const int k0 = tl.start + (int)threadIdx.x * kTilePer;
        unsigned m = 0;
        int n = 0;
        for (int q = 0; q < kTilePer; ++q) {
            const int k = k0 + q;
            if (k < tl.end && is_live(L, tl.list, k)) {
                m |= 1u << q;
                ++n;
            }
        }
        int tot;
        int o = block_excl_scan(n, s_w, tot) + reg[2 * tl.region] + tile_off[b] - tile_off[reg_first[tl.region]];
        int* out = tl.list == 0 ? out_ni : (tl.list == 1 ? out_nj : out_tri);
        for (int q = 0; q < kTilePer; ++q)
            if (m >> q & 1) out[o++] = k0 + q;
    }
}

// incremental update, part 1: the elements deleted in the previous step (int4 sweep of del_step)
__device__ __forceinline__ void find_del_body(int bid, int nb, unsigned int* ctl, const int* del_step, int nE, int t,
                                              const double* t_rd, int* dlist) {
    if (ld_ctl(&ctl[kDel]) == 0) return;
    if (t_rd) t = (int)*t_rd + 1;
    const int n4 = nE >> 2;
    const int4* d4 = reinterpret_cast<const int4*>(del_step);
    for (int v = bid * blockDim.x + threadIdx.x; v < n4; v += nb * blockDim.x) {
        const int4 d = d4[v];
        if (d.x == t - 1) dlist[atomicAdd(&ctl[kNdel], 1u)] = 4 * v;
        if (d.y == t - 1) dlist[atomicAdd(&ctl[kNdel], 1u)] = 4 * v + 1;
        if (d.z == t - 1) dlist[atomicAdd(&ctl[kNdel], 1u)] = 4 * v + 2;
        if (d.w == t - 1) dlist[atomicAdd(&ctl[kNdel], 1u)] = 4 * v + 3;
    }
    if (bid == 0 && (int)threadIdx.x < nE - 4 * n4) {
        const int e = 4 * n4 + (int)threadIdx.x;
        if (del_step[e] == t - 1) dlist[atomicAdd(&ctl[kNdel], 1u)] = e;
    }
}

__global__ void k_ct_find_del(unsigned int* ctl, const int* del_step, int nE, int t, const double* t_rd, int* dlist) {
    find_del_body(blockIdx.x, gridDim.x, ctl, del_step, nE, t, t_rd, dlist);
}

// a node entry becomes live with the first deletion among its adders; of several adders deleted in
// the same step, the lowest element id appends it
__device__ __forceinline__ bool newly_live(const int* orig, const int* aptr, const int* add, int k, int e,
                                           const int* del_step, int t) {
    if (orig[k]) return false;
    for (int a = aptr[k]; a < aptr[k + 1]; ++a) {
        const int ad = add[a], st = del_step[ad];
        if (st != 0 && st < t - 1) return false;  // live before (st = -1: deleted before an upload)
        if (st == t - 1 && ad < e) return false;
    }
    return true;
}

struct AppendIn {
    const int *el_tri_ptr, *el_tri, *el_ni_ptr, *el_ni, *el_nj_ptr, *el_nj;
    const int *ni_orig, *ni_aptr, *ni_add, *ni_pair, *nj_orig, *nj_aptr, *nj_add, *nj_pair;
    const int* pair_reg;  // [npairs][2] region of (pair, side), -1 if none
    int tri_reg;
};

// incremental update, part 2: one block per deleted element, one thread per entry its deletion
// exposes (triangles, then i-node entries, then j-node entries)
// (lanes lt of lsz per deleted element: a workgroup, or a wave of a one-workgroup kernel)
__device__ __forceinline__ void append_body(int bid, int nb, unsigned int* ctl, const int* dlist, const AppendIn& A,
                                            const int* del_step, int t, const double* t_rd, int* reg, int* ni_live,
                                            int* nj_live, int* tri_live, int lt, int lsz) {
    if (ld_ctl(&ctl[kDel]) == 0) return;
    if (t_rd) t = (int)*t_rd + 1;
    const int nd = (int)ld_ctl(&ctl[kNdel]);
    for (int q = bid; q < nd; q += nb) {
        const int e = dlist[q];
        const int t0 = A.el_tri_ptr[e], nt = A.el_tri_ptr[e + 1] - t0;
        const int i0 = A.el_ni_ptr[e], ni = A.el_ni_ptr[e + 1] - i0;
        const int j0 = A.el_nj_ptr[e], nj = A.el_nj_ptr[e + 1] - j0;
        for (int x = lt; x < nt + ni + nj; x += lsz) {
            if (x < nt) {  // unique adder per triangle
                tri_live[atomicAdd(&reg[2 * A.tri_reg + 1], 1)] = A.el_tri[t0 + x];
            } else if (x < nt + ni) {
                const int k = A.el_ni[i0 + x - nt];
                if (!newly_live(A.ni_orig, A.ni_aptr, A.ni_add, k, e, del_step, t)) continue;
                const int r = A.pair_reg[2 * A.ni_pair[k]];
                ni_live[reg[2 * r] + atomicAdd(&reg[2 * r + 1], 1)] = k;
            } else {
                const int k = A.el_nj[j0 + x - nt - ni];
                if (!newly_live(A.nj_orig, A.nj_aptr, A.nj_add, k, e, del_step, t)) continue;
                const int r = A.pair_reg[2 * A.nj_pair[k] + 1];
                nj_live[reg[2 * r] + atomicAdd(&reg[2 * r + 1], 1)] = k;
            }
        }
    }
}

__global__ void k_ct_append(unsigned int* ctl, const int* dlist, AppendIn A, const int* del_step, int t,
                            const double* t_rd, int* reg, int* ni_live, int* nj_live, int* tri_live) {
    append_body(blockIdx.x, gridDim.x, ctl, dlist, A, del_step, t, t_rd, reg, ni_live, nj_live, tri_live,
                (int)threadIdx.x, (int)blockDim.x);
}

// bounding boxes of the live node lists per pair (:2281-2299). Segment = the live node entries of
// one pair side. kSegBlocks blocks per segment reduce in registers, then across the block
// (shuffles + LDS), then issue ONE atomic per bound.
constexpr int kSegBlocks = 256;

struct Seg {
    int start, end, pair, side;  // side 0: i-nodes, 1: j-nodes
    int region;
    int dup;       // 1: the same live node set as an earlier segment, whose boxes also fill this one's
    int alias[2];  // bbox offsets (12 pair + 6 side) of up to two such duplicates, -1 if none
};

__device__ __forceinline__ unsigned long long umin64(unsigned long long a, unsigned long long b) { return a < b ? a : b; }
__device__ __forceinline__ unsigned long long umax64(unsigned long long a, unsigned long long b) { return a > b ? a : b; }

// segment vb / sb, part vb % sb
__device__ __forceinline__ void bbox_body(int vb, int sb, const StepIn& s, const Seg* segs, const int* reg,
                                          const int* ni_live, const int* nj_live, const int* ni_node,
                                          const int* nj_node, unsigned long long* bbox) {
    const Seg sg = segs[vb / sb];
    if (sg.dup) return;  // another segment's blocks fill its boxes
    const int sub = vb % sb;
    const bool side_i = sg.side == 0;
    const int* node = side_i ? ni_node : nj_node;
    const int* lst = (side_i ? ni_live : nj_live) + reg[2 * sg.region];
    const int cnt = reg[2 * sg.region + 1];
    const int bd = (int)blockDim.x;
    unsigned long long mn[3] = {~0ULL, ~0ULL, ~0ULL}, mx[3] = {0ULL, 0ULL, 0ULL};
#pragma unroll 4
    for (int q = sub * bd + (int)threadIdx.x; q < cnt; q += sb * bd) {  // iterations overlap their loads
        double p[3];
        pos(s, node[lst[q]], p);
        for (int d = 0; d < 3; ++d) {
            const unsigned long long e = enc(p[d]);
            mn[d] = umin64(mn[d], e);
            mx[d] = umax64(mx[d], e);
        }
    }
    for (int off = 32; off > 0; off >>= 1)
        for (int d = 0; d < 3; ++d) {
            mn[d] = umin64(mn[d], __shfl_xor(mn[d], off));
            mx[d] = umax64(mx[d], __shfl_xor(mx[d], off));
        }
    __shared__ unsigned long long red[16][6];
    const int w = threadIdx.x / 64;
    if ((threadIdx.x & 63) == 0)
        for (int d = 0; d < 3; ++d) {
            red[w][d] = mn[d];
            red[w][3 + d] = mx[d];
        }
    __syncthreads();
    if (threadIdx.x < 6) {
        const int q = threadIdx.x;
        unsigned long long v = red[0][q];
        for (int ww = 1; ww < bd / 64; ++ww) v = q < 3 ? umin64(v, red[ww][q]) : umax64(v, red[ww][q]);
        for (int a = -1; a < 2; ++a) {  // own slot, then the duplicates'
            const int off = a < 0 ? 12 * sg.pair + (side_i ? 0 : 6) : sg.alias[a];
            if (off < 0) continue;
            unsigned long long* bb = bbox + off;
            if (q < 3) {
                if (v != ~0ULL) atomicMin(&bb[q], v);
            } else if (v != 0ULL) {
                atomicMax(&bb[q], v);
            }
        }
    }
}

__global__ __launch_bounds__(kB) void k_ct_bbox(StepIn s, const Seg* segs, const int* reg, const int* ni_live,
                                                const int* nj_live, const int* ni_node, const int* nj_node,
                                                unsigned long long* bbox, int sb) {
    bbox_body(blockIdx.x, sb, s, segs, reg, ni_live, nj_live, ni_node, nj_node, bbox);
}

// the hash record of live i-node nd (local id) of pair pr at position p inside the range box r
__device__ __forceinline__ void bin_rec(const StepIn& s, const Range& r, const PairParam& pp, int pr, int nd,
                                        const double p[3], BRec& e) {
#pragma clang fp contract(off)
    for (int d = 0; d < 3; ++d) e.e.m[d] = (long long)ceil((p[d] - r.amn[d]) / pp.ddiv);
    const int g = gid(s, nd);
    e.e.node = g;
    e.e.pad = pr;
    for (int d = 0; d < 3; ++d) e.e.p[d] = p[d];
    e.e.next = -1;
    velo(s, nd, e.w.v);
    e.w.mq = s.mass[g / 3];  // diag_M[i] with the node id i (:2592)
}

// entry `slot` of the bucket list into bucket b of search sequence seq: pushed onto the bucket's
// chain (the order of a bucket's entries is the atomics' and irrelevant: every event's force is
// summed order-independently)
__device__ __forceinline__ void bucket_push(unsigned long long* head, int b, unsigned seq, int slot, BEnt e, BVel w,
                                            BEnt* blist, BVel* bvel) {
    const unsigned long long old = atomicExch(&head[b], ((unsigned long long)seq << 32) | (unsigned)slot);
    e.next = (unsigned)(old >> 32) == seq ? (long long)(unsigned)old : -1LL;
    blist[slot] = e;
    bvel[slot] = w;
}

// cells of the live i-nodes inside the pair's range box (:2333-2346) -> the hash grid, each binned
// node at its live-list position in the bucket list. vb = virtual block (segment vb / sb, part
// vb % sb); a launch of nseg * sb workgroups has one each.
__device__ __forceinline__ void bin_body(int vb, const StepIn& s, const Seg* segs, const int* reg, const int* ni_live,
                                         const int* ni_pair, const int* ni_node, const PairParam* par,
                                         const unsigned long long* bbox, const unsigned int* ctl,
                                         unsigned long long* head, BEnt* blist, BVel* bvel, int sb) {
#pragma clang fp contract(off)
    const Seg sg = segs[vb / sb];
    if (sg.side != 0) return;
    const int base = reg[2 * sg.region], n = reg[2 * sg.region + 1];
    const int bd = (int)blockDim.x;
    const unsigned seq = ctl[kSeq];
    for (int q = (vb % sb) * bd + (int)threadIdx.x; q < n; q += sb * bd) {
        const int k = ni_live[base + q];
        const int pr = ni_pair[k];
        const Range r = pair_range(bbox + 12 * pr);
        const int nd = ni_node[k];
        const PairParam pp = par[pr];  // loaded with the box, not behind the range test
        double p[3];
        pos(s, nd, p);
        if (r.empty || p[0] < r.mn[0] || p[1] < r.mn[1] || p[2] < r.mn[2] || p[0] > r.mx[0] || p[1] > r.mx[1] ||
            p[2] > r.mx[2])  // the candidate test of :2514-2519, applied before binning
            continue;
        BRec e;
        bin_rec(s, r, pp, pr, nd, p, e);
        const int b = pp.hash_off + (int)(hash3(e.e.m[0], e.e.m[1], e.e.m[2]) & (unsigned)(pp.hash_size - 1));
        bucket_push(head, b, seq, base + q, e.e, e.w, blist, bvel);  // coalesced by live position
    }
}

__global__ __launch_bounds__(kB) void k_ct_bin(StepIn s, const Seg* segs, const int* reg, const int* ni_live,
                                               const int* ni_pair, const int* ni_node, const PairParam* par,
                                               const unsigned long long* bbox, const unsigned int* ctl,
                                               unsigned long long* head, BEnt* blist, BVel* bvel, int sb) {
    bin_body(blockIdx.x, s, segs, reg, ni_live, ni_pair, ni_node, par, bbox, ctl, head, blist, bvel, sb);
}

// wave-aggregated append: one atomic per wave; every lane of the wave must call it
__device__ __forceinline__ unsigned wave_append(unsigned int* ctr, bool pred) {
    const unsigned long long m = __ballot(pred);
    const int lane = (int)(threadIdx.x & 63);
    const int leader = m ? __ffsll((long long)m) - 1 : 0;
    unsigned base = 0;
    if (m && lane == leader) base = atomicAdd(ctr, (unsigned)__popcll(m));
    base = __shfl(base, leader);
    return base + (unsigned)__popcll(m & ((1ULL << lane) - 1ULL));
}

// Same with one global atomic per BLOCK (the per-wave atomics of a large grid on one counter
// serialise): every thread of the block must call it (block-uniform trip counts).
__device__ __forceinline__ unsigned block_append(unsigned int* ctr, bool pred, unsigned* s_ctl) {
    if (threadIdx.x == 0) s_ctl[0] = 0;
    __syncthreads();
    const unsigned long long m = __ballot(pred);
    const int lane = (int)(threadIdx.x & 63);
    const int leader = m ? __ffsll((long long)m) - 1 : 0;
    unsigned off = 0;
    if (m && lane == leader) off = atomicAdd(&s_ctl[0], (unsigned)__popcll(m));
    off = __shfl(off, leader);
    __syncthreads();
    if (threadIdx.x == 0) s_ctl[1] = s_ctl[0] ? atomicAdd(ctr, s_ctl[0]) : 0u;
    __syncthreads();
    return s_ctl[1] + off + (unsigned)__popcll(m & ((1ULL << lane) - 1ULL));
}

// The same for two counts per thread packed in one 64-bit value (low and high 32 bits; a block's
// sums stay below 2^32 each), appended to one 64-bit counter with one atomic per block: the
// thread's first slots, packed (every thread of the block calls it)
__device__ __forceinline__ unsigned long long block_append2(unsigned long long* ctr, unsigned long long v,
                                                            unsigned long long* s_ctl) {
    if (threadIdx.x == 0) s_ctl[0] = 0;
    __syncthreads();
    const int lane = (int)(threadIdx.x & 63);
    unsigned long long x = v;  // wave inclusive scan
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned long long y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    unsigned long long woff = 0;
    const unsigned long long wtot = __shfl(x, 63);
    if (lane == 63 && wtot) woff = atomicAdd(&s_ctl[0], wtot);
    woff = __shfl(woff, 63);
    __syncthreads();
    if (threadIdx.x == 0) s_ctl[1] = s_ctl[0] ? atomicAdd(ctr, s_ctl[0]) : 0ULL;
    __syncthreads();
    return s_ctl[1] + woff + x - v;
}

// Prefix of 64 shard counters (each clamped to the shard capacity) in LDS, one lane per shard of
// wave 0 (one load and a wave scan, not 64 dependent loads on one thread): s_pre[0..64] = prefix,
// s_pre[65] = some shard overflowed, s_pre[66] = raw total, s_pre[67] = largest shard. Returns the
// clamped total. s_pre holds 68 entries.
__device__ __forceinline__ long long shard_scan(const unsigned int* cnts, long long shard_cap, unsigned* s_pre) {
    if (threadIdx.x < 64) {
        const int q = (int)threadIdx.x;
        const unsigned v = cnts[q * kShardStride];
        const unsigned cl = (long long)v < shard_cap ? v : (unsigned)shard_cap;
        unsigned x = cl, raw = v, mx = v;
        for (int o = 1; o < 64; o <<= 1) {
            const unsigned y = __shfl_up(x, o);
            if (q >= o) x += y;
            raw += __shfl_xor(raw, o);
            mx = max(mx, __shfl_xor(mx, o));
        }
        s_pre[q] = x - cl;
        const bool over = __any((long long)v > shard_cap);
        if (q == 63) {
            s_pre[64] = x;
            s_pre[65] = over ? 1u : 0u;
            s_pre[66] = raw;
            s_pre[67] = mx;
        }
    }
    __syncthreads();
    return s_pre[64];
}

// index in shard-prefix order -> slot of the shard buffers
__device__ __forceinline__ long long shard_slot(const unsigned* s_pre, long long shard_cap, long long ev) {
    int lo = 0, hi = kEvShards;  // s_pre[lo] <= ev < s_pre[hi]
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if ((long long)s_pre[mid] <= ev) lo = mid; else hi = mid;
    }
    return (long long)lo * shard_cap + (ev - s_pre[lo]);
}

// Per-candidate triangle record, written by the prefilter: everything of the loop body at
// :2371-2698 that does not depend on the contact point (same expressions as the reference, so the
// same bits), so the per-cell threads start from one load instead of a chain of dependent ones.
struct TriRec {
    double q0[3], c[3], Rmax, n[3], vdet, im[9], kk;
    double vj[3];  // velocity of the triangle's first node (the event's relative velocity, :2580-2582)
    long long mj[3];
    int j0, j1, j2, eleid, pr;  // global node ids; eleid: the (local) element, for the self-contact test
    int hoff, hmask, self;  // the pair's hash region and self-contact flag (no parameter load in the search)
};

__device__ __forceinline__ void tri_geom(int pr, const Range& r, const PairParam& pp, int nd0, int nd1, int nd2,
                                         int ele, const double q0[3], const double q1[3], const double q2[3],
                                         const double vj[3], TriRec& T) {
#pragma clang fp contract(off)
    const double cx = (q0[0] + q1[0] + q2[0]) / 3.0, cy = (q0[1] + q1[1] + q2[1]) / 3.0,
                 cz = (q0[2] + q1[2] + q2[2]) / 3.0;
    const double R0 = my3norm(q0[0] - cx, q0[1] - cy, q0[2] - cz);
    const double R1 = my3norm(q1[0] - cx, q1[1] - cy, q1[2] - cz);
    const double R2 = my3norm(q2[0] - cx, q2[1] - cy, q2[2] - cz);
    const double v1x = q1[0] - q0[0], v1y = q1[1] - q0[1], v1z = q1[2] - q0[2];
    const double v2x = q2[0] - q0[0], v2y = q2[1] - q0[1], v2z = q2[2] - q0[2];
    const double L1 = my3norm(v1x, v1y, v1z), L2 = my3norm(v2x, v2y, v2z);
    const double Lmax = fmax(L1, L2);
    double nx = v1y * v2z - v1z * v2y, ny = v1z * v2x - v1x * v2z, nz = v1x * v2y - v1y * v2x;  // my3crossNNz
    const double mag_n = sqrt(nx * nx + ny * ny + nz * nz);
    nx = nx / mag_n;
    ny = ny / mag_n;
    nz = nz / mag_n;
    const double d12 = v1x * v2x + v1y * v2y + v1z * v2z;
    const double S = 0.5 * sqrt(L1 * L1 * L2 * L2 - d12 * d12);
    const double A11 = v1x, A21 = v1y, A31 = v1z, A12 = v2x, A22 = v2y, A32 = v2z, A13 = -nx, A23 = -ny, A33 = -nz;
    // my3SolveAb (:3342-3373): determinant and adjugate do not depend on the point
    T.vdet = (A11 * A22 * A33 + A12 * A23 * A31 + A13 * A21 * A32 - A11 * A23 * A32 - A12 * A21 * A33 -
              A13 * A22 * A31);
    T.im[0] = A22 * A33 - A23 * A32;  // im11
    T.im[1] = A13 * A32 - A12 * A33;  // im12
    T.im[2] = A12 * A23 - A13 * A22;  // im13
    T.im[3] = A23 * A31 - A21 * A33;  // im21
    T.im[4] = A11 * A33 - A13 * A31;  // im22
    T.im[5] = A13 * A21 - A11 * A23;  // im23
    T.im[6] = A21 * A32 - A22 * A31;  // im31
    T.im[7] = A12 * A31 - A11 * A32;  // im32
    T.im[8] = A11 * A22 - A12 * A21;  // im33
    T.kk = pp.young * S / Lmax * pp.kc;  // :2575
    for (int d = 0; d < 3; ++d) {
        T.q0[d] = q0[d];
        T.mj[d] = (long long)ceil((q0[d] - r.amn[d]) / pp.ddiv);
    }
    T.c[0] = cx;
    T.c[1] = cy;
    T.c[2] = cz;
    T.Rmax = fmax(fmax(R0, R1), R2);
    T.n[0] = nx;
    T.n[1] = ny;
    T.n[2] = nz;
    T.j0 = nd0;
    T.j1 = nd1;
    T.j2 = nd2;
    T.eleid = ele;
    T.vj[0] = vj[0];
    T.vj[1] = vj[1];
    T.vj[2] = vj[2];
    T.pr = pr;
    T.hoff = pp.hash_off;
    T.hmask = pp.hash_size - 1;
    T.self = pp.self ? 1 : 0;
}

// Which cells dc (0..26: dx fastest, the reference's dz, dy, dx loops) of the 27 around the
// candidate's first-node cell can hold an i-node within the candidate's sphere (|p - c| < Rmax,
// :2532-2536)? A node lies in cell m when ceil((p - amn) / ddiv) == m (bin_rec), i.e. p in
// (amn + (m-1) ddiv, amn + m ddiv] up to the rounding of that expression. Each box is widened by far
// more than that rounding and the radius by a relative 1e-9, so a cell is dropped only if no node
// in it can pass the sphere test: the search visits fewer cells and finds the same events. The
// squared distance is separable, 3 per axis; NaN geometry keeps every cell. Returns a 27-bit mask.
__device__ __forceinline__ unsigned reach_mask(const TriRec& T, const double amn[3], double ddiv) {
    double t2[3][3];
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double m = (double)(T.mj[d] + (k - 1));
            const double eps = 1e-9 * ddiv + 1e-12 * (fabs(amn[d]) + fabs(m) * ddiv);
            const double lo = amn[d] + (m - 1.0) * ddiv - eps, hi = amn[d] + m * ddiv + eps;
            const double t = fmax(fmax(lo - T.c[d], T.c[d] - hi), 0.0);
            t2[d][k] = t * t;
        }
    const double r = T.Rmax * (1.0 + 1e-9) + 1e-9 * ddiv;
    const double r2 = r * r * (1.0 + 1e-9);
    unsigned mask = 0;
#pragma unroll
    for (int dc = 0; dc < 27; ++dc)
        if (!(t2[0][dc % 3] + t2[1][(dc / 3) % 3] + t2[2][dc / 9] > r2)) mask |= 1u << dc;
    return mask;
}

// The full prefilter test (:2374-2411) of live triangle j of pair pr with range box r (act: a real
// entry; every thread of the block calls it): active element, not entirely on one side of the range
// box along any axis -> candidate record in the block's shard (multi-GPU: a rank's lists hold the
// triangles of its own elements only) and one search item per cell of its neighbourhood that its
// sphere can reach (reach_mask)
__device__ __forceinline__ void tri_test(int bid, const StepIn& s, int j, int pr, const Range& r, bool act,
                                         const int* tri_nodes, const int* tri_ele, const PairParam* par,
                                         unsigned int* ccnt, TriRec* cand, long long cshard_cap, uint2* item,
                                         unsigned long long* s_app) {
#pragma clang fp contract(off)
    // every load issued up front (inactive lanes re-read a real entry)
    const int ele = tri_ele[j];
    const int nd0 = tri_nodes[3 * j], nd1 = tri_nodes[3 * j + 1], nd2 = tri_nodes[3 * j + 2];
    const int fl = s.flag[ele];
    const PairParam pp = par[pr];
    double p0[3], p1[3], p2[3];
    pos(s, nd0, p0);
    pos(s, nd1, p1);
    pos(s, nd2, p2);
    bool keep = act && fl == 1;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        keep &= !(p0[d] < r.mn[d] && p1[d] < r.mn[d] && p2[d] < r.mn[d]);
        keep &= !(p0[d] > r.mx[d] && p1[d] > r.mx[d] && p2[d] > r.mx[d]);
    }
    TriRec T;
    unsigned mask = 0u;
    if (keep) {
        double vj[3];
        velo(s, nd0, vj);
        tri_geom(pr, r, pp, gid(s, nd0), gid(s, nd1), gid(s, nd2), ele, p0, p1, p2, vj, T);
        if (item) mask = reach_mask(T, r.amn, pp.ddiv);  // (small decks: no items, k_ct_tri32)
    }
    const unsigned ni = (unsigned)__popc(mask);
    // the candidate and its items appended with ONE atomic per block (the shard's two counters are
    // one 64-bit word: candidates low, items high)
    const int shard = bid % kCandShards;
    const unsigned long long at = block_append2(
        reinterpret_cast<unsigned long long*>(&ccnt[shard * kShardStride]), (keep ? 1ULL : 0ULL) | (unsigned long long)ni << 32,
        s_app);
    const unsigned slot = (unsigned)at;
    const bool stored = keep && (long long)slot < cshard_cap;
    if (stored) cand[shard * cshard_cap + slot] = T;
    if (ni) {
        const long long icap = kItemsPerCand * cshard_cap;
        uint2* out = item + (long long)shard * icap;
        unsigned it = (unsigned)(at >> 32);
        // (a candidate past its shard fails the step -- kCandOver poisons it -- but its items must
        // still name a real record: the shard's first)
        const unsigned cs = (unsigned)(shard * cshard_cap + (stored ? slot : 0u));
        for (unsigned mm = mask; mm; mm &= mm - 1) {
            const int dc = __ffs(mm) - 1;
            const unsigned b = (unsigned)T.hoff + (hash3(T.mj[0] + (dc % 3 - 1), T.mj[1] + ((dc / 3) % 3 - 1),
                                                         T.mj[2] + (dc / 9 - 1)) & (unsigned)T.hmask);
            if ((long long)it < icap) out[it] = make_uint2(cs, ((unsigned)dc << 27) | b);
            ++it;
        }
    }
}

// triangle prefilter over the live triangles, one per thread: the full test
__device__ __forceinline__ void tri_filter_body(int bid, int nb, const StepIn& s, const int* tri_cnt,
                                                const int* tri_live, const int* tri_pair, const int* tri_nodes,
                                                const int* tri_ele, const PairParam* par,
                                                const unsigned long long* bbox, unsigned int* ccnt, TriRec* cand,
                                                long long cshard_cap, uint2* item) {
    const int n = *tri_cnt;
    __shared__ unsigned long long s_app[2];
    const int tid = (int)threadIdx.x;
    unsigned* tested = &ccnt[(bid % kCandShards) * kShardStride + kTestWord];
    for (int q0 = bid * kB; q0 < n; q0 += nb * kB) {  // block-uniform trip count
        const int q = q0 + tid;
        const int j = tri_live[q < n ? q : n - 1];
        const int pr = tri_pair[j];
        const Range r = pair_range(bbox + 12 * pr);
        const bool act = q < n && !r.empty;
        const unsigned long long m = __ballot(act);
        if ((tid & 63) == 0 && m) atomicAdd(tested, (unsigned)__popcll(m));
        tri_test(bid, s, j, pr, r, act, tri_nodes, tri_ele, par, ccnt, cand, cshard_cap, item, s_app);
    }
}

__global__ __launch_bounds__(kB) void k_ct_tri_filter(StepIn s, const int* tri_cnt, const int* tri_live,
                                                      const int* tri_pair, const int* tri_nodes, const int* tri_ele,
                                                      const PairParam* par, const unsigned long long* bbox,
                                                      unsigned int* ccnt, TriRec* cand, long long cshard_cap,
                                                      uint2* item) {
    tri_filter_body(blockIdx.x, gridDim.x, s, tri_cnt, tri_live, tri_pair, tri_nodes, tri_ele, par, bbox, ccnt, cand,
                    cshard_cap, item);
}

// events of one thread, kept in registers and appended with one atomic per wave (a same-address
// atomic per event serialised the kernel); more than kEvLocal go out one by one
constexpr int kEvLocal = 4;
struct EvBuf {
    int n, j0, j1, j2;
    int i[kEvLocal];
    double f[kEvLocal][3];
};

__device__ __forceinline__ void ev_write(int* ev_nodes, double* ev_f, long long e, int i, int j0, int j1, int j2,
                                         double fx, double fy, double fz) {
    int* en = ev_nodes + 4 * e;
    en[0] = i;
    en[1] = j0;
    en[2] = j1;
    en[3] = j2;
    double* ef = ev_f + 3 * e;
    ef[0] = fx;
    ef[1] = fy;
    ef[2] = fz;
}

// one bucket entry: its four 16-B vectors are issued together and pinned (the asm), so the
// compiler cannot split the record into per-field loads sunk behind the tests that use them --
// that made every entry a chain of four dependent round trips
__device__ __forceinline__ long long ll2(unsigned lo, unsigned hi) {
    return (long long)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ BEnt ld_bent(const BEnt* e) {
    const uint4* q = reinterpret_cast<const uint4*>(e);
    const uint4 w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
    asm volatile("" ::"v"(w0.x), "v"(w1.x), "v"(w2.x), "v"(w3.x));
    BEnt r;
    r.m[0] = ll2(w0.x, w0.y);
    r.m[1] = ll2(w0.z, w0.w);
    r.m[2] = ll2(w1.x, w1.y);
    r.node = (int)w1.z;
    r.pad = (int)w1.w;
    r.p[0] = __longlong_as_double(ll2(w2.x, w2.y));
    r.p[1] = __longlong_as_double(ll2(w2.z, w2.w));
    r.p[2] = __longlong_as_double(ll2(w3.x, w3.y));
    r.next = ll2(w3.z, w3.w);
    return r;
}

// one (candidate triangle, neighbour cell) pair: the rest of the loop body at :2371-2698 for the
// i-nodes of cell mj (one of the 27 around the triangle's first node), found in hash bucket b.
template <bool EXACT_CELL>
__device__ __forceinline__ void tri_cell(const StepIn& s, const TriRec* __restrict__ rec, const long long mj[3],
                                         int b, unsigned seq, const PairParam* par, const unsigned long long* head,
                                         const BEnt* __restrict__ blist, const BVel* __restrict__ bvel, double d_lim,
                                         double myu, unsigned int* evn, long long cap, int* ev_nodes, double* ev_f,
                                         EvBuf& eb) {
#pragma clang fp contract(off)
    const int pr = rec->pr;
    const unsigned long long h = head[b];
    const int first = (unsigned)(h >> 32) == seq ? (int)(unsigned)h : -1;  // an older stamp: empty
    // self contact: the triangle's element's own nodes are skipped (:2496-2507); loaded once
    const bool self = rec->self;
    int own8[8];
    if (self) {
        const int* cn = s.conn + 8 * (long long)rec->eleid;
#pragma unroll
        for (int a = 0; a < 8; ++a) own8[a] = gid(s, cn[a]);
    }
    // the point-independent part of the test, held in registers for the whole bucket
    const double c0 = rec->c[0], c1 = rec->c[1], c2 = rec->c[2], Rmax = rec->Rmax;
    const double q00 = rec->q0[0], q01 = rec->q0[1], q02 = rec->q0[2], vdet = rec->vdet;
    double im[9];
#pragma unroll
    for (int k = 0; k < 9; ++k) im[k] = rec->im[k];
    int nxt = -1;
    for (int sl = first; sl >= 0; sl = nxt) {
        const BEnt be = ld_bent(blist + sl);
        nxt = (int)be.next;
        const int i = be.node;
        // branch-free cell and self tests: no load waits behind a branch. EXACT_CELL (search items):
        // only the bucket's entries of this very cell (other cells' entries are found through their
        // own item, if their cell is searched at all); else (32 lanes per candidate, each bucket
        // visited once) every entry of the 27-neighbourhood of the first-node cell mj
        bool skip = EXACT_CELL
                        ? ((int)(mj[0] != be.m[0]) | (int)(mj[1] != be.m[1]) | (int)(mj[2] != be.m[2])) != 0
                        : ((int)(llabs(mj[0] - be.m[0]) > 1) | (int)(llabs(mj[1] - be.m[1]) > 1) |
                           (int)(llabs(mj[2] - be.m[2]) > 1)) != 0;
        if (self) {
#pragma unroll
            for (int a = 0; a < 8; ++a) skip |= (i == own8[a]);
        }
        if (skip) continue;
        const double p[3] = {be.p[0], be.p[1], be.p[2]};
        const double dpc = my3norm(p[0] - c0, p[1] - c1, p[2] - c2);
        if (dpc >= Rmax) continue;
        const double bx = p[0] - q00, by = p[1] - q01, bz = p[2] - q02;
        const double x1 = (im[0] * bx + im[1] * by + im[2] * bz) / vdet;
        const double x2 = (im[3] * bx + im[4] * by + im[5] * bz) / vdet;
        const double d = (im[6] * bx + im[7] * by + im[8] * bz) / vdet;
        if (!(0.0 <= x1 && 0.0 <= x2 && x1 + x2 <= 1.0 && d > 0.0 && d <= d_lim)) continue;
        const int j0 = rec->j0, j1 = rec->j1, j2 = rec->j2;
        const double nx = rec->n[0], ny = rec->n[1], nz = rec->n[2], kk = rec->kk;
        // velo = d_disp / d_time of the previous step (:628), the IC before step 1: formed by the
        // binning (i) and the prefilter (j0)
        const BVel w = bvel[sl];
        const double vx = w.v[0] - rec->vj[0], vy = w.v[1] - rec->vj[1], vz = w.v[2] - rec->vj[2];
        const double mag_v = my3norm(vx, vy, vz);
        double vex = 0.0, vey = 0.0, vez = 0.0;
        if (mag_v > 0.0) {
            vex = vx / mag_v;
            vey = vy / mag_v;
            vez = vz / mag_v;
        }
        const double F = kk * d;
        double fx = F * nx, fy = F * ny, fz = F * nz;
        // damping: diag_M[i] indexes the dof vector with a node id (:2592)
        const double Cd = 2 * sqrt(w.mq * kk) * par[pr].Cr;
        const double fc_x = -Cd * vx, fc_y = -Cd * vy, fc_z = -Cd * vz;
        const double dot_ve_n = vex * nx + vey * ny + vez * nz;
        const double vsx = vex - dot_ve_n * nx, vsy = vey - dot_ve_n * ny, vsz = vez - dot_ve_n * nz;
        const double fric_x = -myu * F * vsx, fric_y = -myu * F * vsy, fric_z = -myu * F * vsz;
        fx += fric_x + fc_x;
        fy += fric_y + fc_y;
        fz += fric_z + fc_z;
        if (eb.n < kEvLocal) {
            eb.j0 = j0;
            eb.j1 = j1;
            eb.j2 = j2;
#pragma unroll
            for (int u = 0; u < kEvLocal; ++u)
                if (u == eb.n) {
                    eb.i[u] = i;
                    eb.f[u][0] = fx;
                    eb.f[u][1] = fy;
                    eb.f[u][2] = fz;
                }
            ++eb.n;
        } else {  // evn: this wave's shard counter, cap: the shard's capacity, ev_*: the shard's slots
            const unsigned e = atomicAdd(evn, 1u);
            if ((long long)e < cap) ev_write(ev_nodes, ev_f, e, i, j0, j1, j2, fx, fy, fz);
        }
    }
}

// the wave's buffered events -> its event shard, one atomic per wave (every lane calls it)
__device__ __forceinline__ void ev_flush(const EvBuf& eb, int lane, unsigned int* evn, long long shard_cap,
                                         int* sh_nodes, double* sh_f) {
    const int c = eb.n < kEvLocal ? eb.n : kEvLocal;
    int x = c;  // wave inclusive scan of the buffered counts
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (__builtin_amdgcn_readlane(x, 63) == 0) return;  // wave-uniform: no events
    unsigned base = 0;
    if (lane == 63) base = atomicAdd(evn, (unsigned)x);
    base = __shfl(base, 63) + (unsigned)(x - c);
#pragma unroll
    for (int u = 0; u < kEvLocal; ++u)
        if (u < c && (long long)(base + u) < shard_cap)
            ev_write(sh_nodes, sh_f, base + u, eb.i[u], eb.j0, eb.j1, eb.j2, eb.f[u][0], eb.f[u][1], eb.f[u][2]);
}

// one lane per search item (candidate triangle, cell): the prefilter listed only the cells its
// sphere reaches, so no lane is idle and no bucket needs deduplicating (each item takes its own
// cell's entries)
__device__ __forceinline__ void tri_body(const StepIn& s, unsigned int* ctl, const unsigned int* ccnt,
                                         const TriRec* cand, long long cshard_cap, const uint2* item,
                                         const PairParam* par, const unsigned long long* head, const BEnt* blist,
                                         const BVel* bvel, double d_lim, double myu, unsigned int* evs,
                                         long long shard_cap, int* ev_nodes, double* ev_f) {
    __shared__ unsigned s_cpre[kCandShards + 4], s_ipre[kCandShards + 4];
    (void)shard_scan(ccnt, cshard_cap, s_cpre);
    const long long icap = kItemsPerCand * cshard_cap;
    const long long n = shard_scan(ccnt + kItemWord, icap, s_ipre);
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // totals for the stats, the overflow check and the poison
        ctl[kNcand] = s_cpre[kCandShards + 2];
        atomicMax(&ctl[kNcandMax], s_cpre[kCandShards + 2]);
        atomicMax(&ctl[kCandShardMax], s_cpre[kCandShards + 3]);
        atomicMax(&ctl[kItemShardMax], s_ipre[kCandShards + 3]);  // search items: own buffer, own report
        ctl[kCandOver] = s_cpre[kCandShards + 1] | s_ipre[kCandShards + 1];
    }
    const int lane = (int)(threadIdx.x & 63);
    const unsigned seq = ctl[kSeq];
    const int shard = (int)(((blockIdx.x * blockDim.x + threadIdx.x) >> 6) % kEvShards);
    unsigned int* evn = evs + shard * kShardStride;
    int* sh_nodes = ev_nodes + 4 * (long long)shard * shard_cap;
    double* sh_f = ev_f + 3 * (long long)shard * shard_cap;
    for (long long q0 = blockIdx.x * (long long)blockDim.x; q0 < n; q0 += (long long)gridDim.x * blockDim.x) {
        const long long q = q0 + threadIdx.x;  // wave-uniform trip count (the append below is wave-wide)
        EvBuf eb;
        eb.n = 0;
        eb.j0 = eb.j1 = eb.j2 = 0;
        if (q < n) {
            const uint2 it = item[shard_slot(s_ipre, icap, q)];
            const TriRec* rec = cand + it.x;
            const int dc = (int)(it.y >> 27);
            const long long cell[3] = {rec->mj[0] + (dc % 3 - 1), rec->mj[1] + ((dc / 3) % 3 - 1),
                                       rec->mj[2] + (dc / 9 - 1)};
            tri_cell<true>(s, rec, cell, (int)(it.y & ((1u << 27) - 1u)), seq, par, head, blist, bvel, d_lim, myu,
                           evn, shard_cap, sh_nodes, sh_f, eb);
        }
        ev_flush(eb, lane, evn, shard_cap, sh_nodes, sh_f);
    }
}

__global__ __launch_bounds__(128) void k_ct_tri(StepIn s, unsigned int* ctl, const unsigned int* ccnt,
                                                const TriRec* cand, long long cshard_cap, const uint2* item,
                                                const PairParam* par, const unsigned long long* head,
                                                const BEnt* blist, const BVel* bvel, double d_lim, double myu,
                                                unsigned int* evs, long long shard_cap, int* ev_nodes, double* ev_f) {
    tri_body(s, ctl, ccnt, cand, cshard_cap, item, par, head, blist, bvel, d_lim, myu, evs, shard_cap, ev_nodes, ev_f);
}

// Small decks: 32 lanes per candidate triangle (27 cells used), lane c takes cell c (dz, dy, dx in the
// reference's loop order); a cell whose bucket a lower cell of the same triangle maps to is
// skipped, so every bucket is visited once (buckets compared across lanes, readlane). No search
// items: at a few hundred candidates the prefilter's item pass costs more than idle lanes do.
__global__ __launch_bounds__(128) void k_ct_tri32(StepIn s, unsigned int* ctl, const unsigned int* ccnt,
                                                  const TriRec* cand, long long cshard_cap, const PairParam* par,
                                                  const unsigned long long* head, const BEnt* blist, const BVel* bvel,
                                                  double d_lim, double myu, unsigned int* evs, long long shard_cap,
                                                  int* ev_nodes, double* ev_f) {
    __shared__ unsigned s_cpre[kCandShards + 4];
    const long long n = 32LL * shard_scan(ccnt, cshard_cap, s_cpre);
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // totals for the stats, the overflow check and the poison
        ctl[kNcand] = s_cpre[kCandShards + 2];
        atomicMax(&ctl[kNcandMax], s_cpre[kCandShards + 2]);
        atomicMax(&ctl[kCandShardMax], s_cpre[kCandShards + 3]);
        ctl[kCandOver] = s_cpre[kCandShards + 1];
    }
    const int lane = (int)(threadIdx.x & 63);
    const unsigned seq = ctl[kSeq];
    const int shard = (int)(((blockIdx.x * blockDim.x + threadIdx.x) >> 6) % kEvShards);
    unsigned int* evn = evs + shard * kShardStride;
    int* sh_nodes = ev_nodes + 4 * (long long)shard * shard_cap;
    double* sh_f = ev_f + 3 * (long long)shard * shard_cap;
    for (long long q0 = blockIdx.x * (long long)blockDim.x; q0 < n; q0 += (long long)gridDim.x * blockDim.x) {
        const long long q = q0 + threadIdx.x;  // wave-uniform trip count (the append below is wave-wide)
        EvBuf eb;
        eb.n = 0;
        eb.j0 = eb.j1 = eb.j2 = 0;
        const int cell = (int)(q & 31);
        const bool valid = q < n && cell < 27;
        const TriRec* rec = cand + (valid ? shard_slot(s_cpre, cshard_cap, q >> 5) : 0);
        long long mj[3] = {0, 0, 0};
        unsigned hb = 0x80000000u | (unsigned)lane;  // never equal to a real bucket (< 2^31)
        int hoff = 0;
        if (valid) {
            hoff = rec->hoff;
            mj[0] = rec->mj[0];
            mj[1] = rec->mj[1];
            mj[2] = rec->mj[2];
            hb = hash3(mj[0] + (cell % 3 - 1), mj[1] + ((cell / 3) % 3 - 1), mj[2] + (cell / 9 - 1)) &
                 (unsigned)rec->hmask;
        }
        bool dup = false;
        const int half = lane & 32;
#pragma unroll
        for (int c2 = 0; c2 < 26; ++c2) {
            const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)hb, c2);
            const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)hb, 32 + c2);
            dup |= c2 < cell && (half ? hi : lo) == hb;
        }
        if (valid && !dup)
            tri_cell<false>(s, rec, mj, hoff + (int)hb, seq, par, head, blist, bvel, d_lim, myu, evn, shard_cap,
                            sh_nodes, sh_f, eb);
        ev_flush(eb, lane, evn, shard_cap, sh_nodes, sh_f);
    }
}

// the event shards; block 0 also publishes the totals for the overflow check and the stats
static_assert(kEvShards == 64 && kCandShards == 64, "shard_scan: one wave lane per shard");
__device__ __forceinline__ long long shard_prefix(int bid, unsigned int* ctl, const unsigned int* evs,
                                                  long long shard_cap, unsigned* s_pre) {
    const long long n = shard_scan(evs, shard_cap, s_pre);
    if (bid == 0 && threadIdx.x == 0) {
        ctl[kEv] = s_pre[kEvShards + 2];
        atomicMax(&ctl[kEvMax], s_pre[kEvShards + 2]);
        atomicMax(&ctl[kEvShardMax], s_pre[kEvShards + 3]);
    }
    return n;
}


// Per-node gather of the event terms over the nodes that received one ("touched", a compact list
// instead of a pass over all nN nodes): count -> per-node term ranges by a wave-aggregated bump
// allocator (ranges are disjoint; their order is irrelevant) -> scatter -> sum.
// Block 0 also poisons the step when a buffer overflowed in it (events beyond a shard, candidate
// triangles beyond their buffer, a truncated multi-GPU mirror block): the nodal, BC, element and
// interface kernels of this and later steps of the call then write nothing (hakai_kernels.hip,
// poisoned), so the state stays the last good step's and hakai_step reports the overflow.
__device__ __forceinline__ void count_body(int bid, int nb, unsigned int* ctl, const unsigned int* evs,
                                           long long shard_cap, const int* ev_nodes, int* cnt, int* touched,
                                           int* tpos, int tsel, int* poison, int t, const double* t_rd) {
    __shared__ unsigned s_pre[kEvShards + 4];
    const long long n = 4 * shard_prefix(bid, ctl, evs, shard_cap, s_pre);
    if (bid == 0 && threadIdx.x == 0) {
        const bool over = ctl[kCandOver] != 0 || s_pre[kEvShards + 1];
        if (over && poison[0] == 0) {
            poison[1] = t_rd ? (int)*t_rd + 1 : t;
            poison[0] = 1;
        }
    }
    __shared__ unsigned s_app[2];
    for (long long e0 = bid * (long long)blockDim.x; e0 < n; e0 += (long long)nb * blockDim.x) {
        const long long e = e0 + threadIdx.x;
        int node = -1;
        bool first = false;
        if (e < n) {
            node = ev_nodes[4 * shard_slot(s_pre, shard_cap, e >> 2) + (e & 3)];
            first = atomicAdd(&cnt[node], 1) == 0;
        }
        const unsigned q = block_append(&ctl[kTouched + tsel], first, s_app);
        if (first) {
            touched[q] = node;
            tpos[node] = (int)q;
        }
    }
}

__global__ void k_ct_count(unsigned int* ctl, const unsigned int* evs, long long shard_cap, const int* ev_nodes,
                           int* cnt, int* touched, int* tpos, int tsel, int* poison, int t, const double* t_rd) {
    count_body(blockIdx.x, gridDim.x, ctl, evs, shard_cap, ev_nodes, cnt, touched, tpos, tsel, poison, t, t_rd);
}

__device__ __forceinline__ void alloc_body(int bid, int nb, unsigned int* ctl, int tsel, const int* touched,
                                           const int* cnt, int* toff, int* tcnt) {
    const int nt = (int)ld_ctl(&ctl[kTouched + tsel]);
    const int lane = (int)(threadIdx.x & 63);
    for (int q0 = bid * blockDim.x; q0 < nt; q0 += nb * blockDim.x) {
        const int q = q0 + (int)threadIdx.x;
        const int c = q < nt ? cnt[touched[q]] : 0;
        int x = c;  // wave inclusive scan
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        unsigned base = 0;
        if (lane == 63) base = atomicAdd(&ctl[kTerms], (unsigned)x);
        base = __shfl(base, 63);
        if (q < nt) {
            toff[q] = (int)base + x - c;
            tcnt[q] = c;
        }
    }
}

__global__ void k_ct_alloc(unsigned int* ctl, int tsel, const int* touched, const int* cnt, int* toff, int* tcnt) {
    alloc_body(blockIdx.x, gridDim.x, ctl, tsel, touched, cnt, toff, tcnt);
}

__device__ __forceinline__ void scatter_body(int bid, int nb, unsigned int* ctl, const unsigned int* evs,
                                             long long shard_cap, const int* ev_nodes, const double* ev_f,
                                             const int* toff, const int* tpos, int* cnt, double* terms) {
#pragma clang fp contract(off)
    __shared__ unsigned s_pre[kEvShards + 4];
    const long long n = 4 * shard_prefix(bid, ctl, evs, shard_cap, s_pre);
    for (long long e = bid * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)nb * blockDim.x) {
        const long long ev = shard_slot(s_pre, shard_cap, e >> 2);
        const int role = (int)(e & 3);
        const int node = ev_nodes[4 * ev + role];
        const int slot = toff[tpos[node]] + atomicSub(&cnt[node], 1) - 1;  // leaves cnt zeroed
        const double* f = ev_f + 3 * ev;
        double* o = terms + 3 * (long long)slot;
        if (role == 0) {  // c_force3[i] += f
            o[0] = f[0];
            o[1] = f[1];
            o[2] = f[2];
        } else {  // triangle nodes: += -f / 3.0
            o[0] = -f[0] / 3.0;
            o[1] = -f[1] / 3.0;
            o[2] = -f[2] / 3.0;
        }
    }
}

__global__ void k_ct_scatter(unsigned int* ctl, const unsigned int* evs, long long shard_cap, const int* ev_nodes,
                             const double* ev_f, const int* toff, const int* tpos, int* cnt, double* terms) {
    scatter_body(blockIdx.x, gridDim.x, ctl, evs, shard_cap, ev_nodes, ev_f, toff, tpos, cnt, terms);
}

// external_force = 0.0 + (sum of the node's terms), summed in double-double and rounded once
__device__ __forceinline__ void sum_body(int bid, int nb, const unsigned int* ctl, int tsel, const int* touched,
                                         const int* toff, const int* tcnt, const double* terms, double* fext,
                                         const int* g2l = nullptr) {
#pragma clang fp contract(off)
    const int nt = (int)ld_ctl(&ctl[kTouched + tsel]);
    for (int q = bid * blockDim.x + threadIdx.x; q < nt; q += nb * blockDim.x) {
        const long long n = g2l ? g2l[touched[q]] : touched[q];
        const int a = toff[q], b = a + tcnt[q];
        for (int c = 0; c < 3; ++c) {
            double s = 0.0, e = 0.0;
            for (int i = a; i < b; ++i) {
                const double x = terms[3 * (long long)i + c];
                const double t = s + x;  // TwoSum
                const double bp = t - s;
                const double err = (s - (t - bp)) + (x - bp);
                s = t;
                e += err;
            }
            fext[3 * n + c] = s + e;
        }
    }
}

__global__ void k_ct_sum(unsigned int* ctl, int tsel, const int* touched, const int* toff, const int* tcnt,
                         const double* terms, double* fext, const int* g2l) {
    sum_body(blockIdx.x, gridDim.x, ctl, tsel, touched, toff, tcnt, terms, fext, g2l);
    // multi-GPU: the next step's touched list starts empty (its steps run no k_ct_reset)
    if (g2l && blockIdx.x == 0 && threadIdx.x == 0) ctl[kTouched + 1 - tsel] = 0;
}

// ---- small decks: fused single-workgroup phases ------------------------------------------------
// The reference's own decks have a few thousand contact entries and tens of events per step, so
// the ~13 launches of a contact step (each >= ~2.4 us from a graph, tools/barrier_probe.hip) cost
// more than their work. For models small at setup (Contact::small) the step runs the prologue
// (reset, deletion scan, surface append) and the event gather (count, alloc, scatter, sum) each as
// ONE 1024-thread workgroup, the bodies separated by workgroup barriers; the binning and the
// triangle prefilter share one launch. Same bodies, same results.
constexpr int kSmallThreads = 1024;

__global__ __launch_bounds__(kSmallThreads) void k_ct_prologue1(
    unsigned long long* bbox, int npairs, unsigned int* ctl, unsigned int* evs, unsigned int* ccnt, const int* del_any,
    int t, const double* t_rd, const int* touched_prev, int tsel, double* fext, const int* del_step, int nE,
    int* dlist, AppendIn A, int* reg, int* ni_live, int* nj_live, int* tri_live, int with_lists) {
    reset_body(0, 1, bbox, npairs, ctl, evs, ccnt, 0, del_any, t, t_rd, touched_prev, tsel, fext);
    if (!with_lists) return;
    __syncthreads();
    find_del_body(0, 1, ctl, del_step, nE, t, t_rd, dlist);
    __syncthreads();
    append_body(0, 1, ctl, dlist, A, del_step, t, t_rd, reg, ni_live, nj_live, tri_live, (int)threadIdx.x,
                (int)blockDim.x);
}

__global__ __launch_bounds__(kSmallThreads) void k_ct_gather1(unsigned int* ctl, const unsigned int* evs,
                                                              long long shard_cap, const int* ev_nodes,
                                                              const double* ev_f, int* cnt, int* touched, int* tpos,
                                                              int tsel, int* poison, int t,
                                                              const double* t_rd, int* toff, int* tcnt,
                                                              double* terms, double* fext) {
    count_body(0, 1, ctl, evs, shard_cap, ev_nodes, cnt, touched, tpos, tsel, poison, t, t_rd);
    __syncthreads();
    alloc_body(0, 1, ctl, tsel, touched, cnt, toff, tcnt);
    __syncthreads();
    scatter_body(0, 1, ctl, evs, shard_cap, ev_nodes, ev_f, toff, tpos, cnt, terms);
    __syncthreads();
    sum_body(0, 1, ctl, tsel, touched, toff, tcnt, terms, fext);
}

// binning (workgroups [0, nbin)) and the triangle prefilter (the rest) in one launch: both need
// only the pair boxes
__global__ __launch_bounds__(kB) void k_ct_binfilter(StepIn s, const Seg* segs, const int* reg, const int* ni_live,
                                                     const int* ni_pair, const int* ni_node, const PairParam* par,
                                                     const unsigned long long* bbox, const unsigned int* ctl,
                                                     unsigned long long* head, BEnt* blist, BVel* bvel,
                                                     int sb, int nbin, const int* tri_cnt,
                                                     const int* tri_live, const int* tri_pair, const int* tri_nodes,
                                                     const int* tri_ele, unsigned int* ccnt, TriRec* cand,
                                                     long long cshard_cap, uint2* item) {
    if ((int)blockIdx.x < nbin)
        bin_body(blockIdx.x, s, segs, reg, ni_live, ni_pair, ni_node, par, bbox, ctl, head, blist, bvel, sb);
    else
        tri_filter_body(blockIdx.x - nbin, gridDim.x - nbin, s, tri_cnt, tri_live, tri_pair, tri_nodes, tri_ele, par,
                        bbox, ccnt, cand, cshard_cap, item);
}

// ---- multi-GPU exchange (hkc::Xrank) --------------------------------------------------------
// Every exchanged block is an int4 header -- (count, overflow, last deletion step, full) -- and its
// records. Rank q's block is read through XBlk.p[q]: the RCCL-gathered receive buffer, or the
// in-process peer's own send buffer (no copy).
using hkc::kMaxXRanks;
using hkc::XBlk;
__device__ __forceinline__ int xhdr(const char* blk, int w) {
    return __hip_atomic_load(reinterpret_cast<const int*>(blk) + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr size_t kXHdr = 16;
constexpr int kNxCount = hkc::Xrank::kNx;

// every rank's block header (count, overflow, last deletion step, full) -> LDS, one lane per rank:
// the loads of all ranks in flight together, not a dependent chain on one thread
__device__ __forceinline__ void load_hdrs(const XBlk& xb, int nr, int4* s_h) {
    const int q = (int)threadIdx.x;
    if (q < nr) {
        const char* b = xb.p[q];
        s_h[q] = make_int4(xhdr(b, 0), xhdr(b, 1), xhdr(b, 2), xhdr(b, 3));
    }
    __syncthreads();
}

struct EvRec {
    int n[4];     // i, j0, j1, j2 (global node ids)
    double f[3];  // force on i (the triangle nodes get -f/3 each)
};

// this rank's events of the step, shard order -> its block; overflow = events beyond a shard or
// candidates beyond their buffer (poisons the step on every rank, k_ct_count_g)
__global__ void k_ev_pack(unsigned int* ctl, const unsigned int* evs, long long shard_cap, const int* ev_nodes,
                          const double* ev_f, char* blk, long long cap) {
    __shared__ unsigned s_pre[kEvShards + 4];
    const long long n = shard_prefix(blockIdx.x, ctl, evs, shard_cap, s_pre);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const bool over = ctl[kCandOver] != 0 || s_pre[kEvShards + 1];
        int* h = reinterpret_cast<int*>(blk);
        h[0] = (int)n;
        h[1] = over ? 1 : 0;
    }
    EvRec* out = reinterpret_cast<EvRec*>(blk + kXHdr);
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n && e < cap;
         e += (long long)gridDim.x * blockDim.x) {
        const long long sl = shard_slot(s_pre, shard_cap, e);
        EvRec r;
        for (int k = 0; k < 4; ++k) r.n[k] = ev_nodes[4 * sl + k];
        for (int k = 0; k < 3; ++k) r.f[k] = ev_f[3 * sl + k];
        out[e] = r;
    }
}

// rank prefix of the blocks' record counts in LDS (each clamped to the block capacity); block 0
// publishes the event total
__device__ __forceinline__ long long rank_prefix(unsigned int* ctl, const int4* s_h, int nr, long long* s_off,
                                                 const int* cap, bool publish) {
    if (threadIdx.x == 0) {
        long long run = 0;
        for (int q = 0; q < nr; ++q) {
            s_off[q] = run;
            run += min(s_h[q].x, cap[q]);
        }
        s_off[nr] = run;
        if (publish && blockIdx.x == 0) {
            ctl[kEv] = (unsigned)run;
            atomicMax(&ctl[kEvMax], (unsigned)run);
        }
    }
    __syncthreads();
    return s_off[nr];
}

__device__ __forceinline__ int rank_of_rec(const long long* s_off, int nr, long long E) {
    int q = 0;
    while (q + 1 < nr && s_off[q + 1] <= E) ++q;
    return q;
}

__device__ __forceinline__ const EvRec* rank_ev(const XBlk& xb, const long long* s_off, int nr, long long E) {
    const int q = rank_of_rec(s_off, nr, E);
    return reinterpret_cast<const EvRec*>(xb.p[q] + kXHdr) + (E - s_off[q]);
}

// any rank's block over its capacity or flagged: poison step pstep on every rank (all read the same
// headers); xctl records which exchange (bit) for the retry
__device__ __forceinline__ void x_overflow_check(const int4* s_h, int nr, const int* cap, int* poison, int pstep,
                                                 int* xctl, int bit) {
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        bool local = false, over = false;  // a rank's own buffers overflowed / the exchange block
        for (int q = 0; q < nr; ++q) {
            local |= s_h[q].y != 0;
            over |= s_h[q].x > cap[q];
        }
        if (over) atomicOr(xctl, bit);
        if (over || local) {
            if (poison[0] == 0) {
                poison[1] = pstep;
                poison[0] = 1;
            }
        }
    }
}

// the gathered record counts of exchange x (a full deletion block counts 0): the step's (read back
// for the capacities two steps later) and their maxima (the growth after an overflow). Recorded by
// the kernel that consumes the blocks, so no pointer to a peer's block outlives its step.
__device__ __forceinline__ void x_counts(const int4* s_h, int nr, int x, int* xctl, int* hc) {
    const int q = (int)threadIdx.x;
    if (blockIdx.x == 0 && blockIdx.y == 0 && q < nr) {
        const int v = (x == 0 && s_h[q].w) ? 0 : s_h[q].x;
        xctl[4 + x * nr + q] = v;
        atomicMax(&xctl[4 + (kNxCount + x) * nr + q], v);
        hc[x * nr + q] = v;  // host-mapped ring slot of the step (no copy launch)
    }
}

// every rank's events; only the terms of this rank's nodes (g2l >= 0) are counted and summed
// (also the reset's share of phase B: the previous step's touched nodes' forces back to 0 -- the
// nodal update of that step has read them -- and the term counter)
__global__ void k_ct_count_g(unsigned int* ctl, XBlk xb, int nr, const int* g2l, int* cnt, int* touched,
                             int* tpos, int tsel, int* poison, int pstep, int* xctl, int* hc, const int* touched_prev,
                             double* fext) {
    __shared__ long long s_off[kMaxXRanks + 1];
    __shared__ unsigned s_app[2];
    __shared__ int4 s_h[kMaxXRanks];
    {
        const int np = (int)ld_ctl(&ctl[kTouched + 1 - tsel]);
        for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < np; q += gridDim.x * blockDim.x) {
            const long long l = g2l[touched_prev[q]];
            fext[3 * l] = 0.0;
            fext[3 * l + 1] = 0.0;
            fext[3 * l + 2] = 0.0;
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) ctl[kTerms] = 0;
    }
    load_hdrs(xb, nr, s_h);
    x_overflow_check(s_h, nr, xb.cap, poison, pstep, xctl, 4);
    x_counts(s_h, nr, 2, xctl, hc);
    const long long n = 4 * rank_prefix(ctl, s_h, nr, s_off, xb.cap, true);
    for (long long e0 = blockIdx.x * (long long)blockDim.x; e0 < n; e0 += (long long)gridDim.x * blockDim.x) {
        const long long e = e0 + threadIdx.x;
        int node = -1;
        bool first = false;
        if (e < n) {
            node = rank_ev(xb, s_off, nr, e >> 2)->n[e & 3];
            first = g2l[node] >= 0 && atomicAdd(&cnt[node], 1) == 0;
        }
        const unsigned q = block_append(&ctl[kTouched + tsel], first, s_app);
        if (first) {
            touched[q] = node;
            tpos[node] = (int)q;
        }
    }
}

__global__ void k_ct_scatter_g(XBlk xb, int nr, const int* g2l, unsigned int* ctl, const int* toff,
                               const int* tpos, int* cnt, double* terms) {
#pragma clang fp contract(off)
    __shared__ long long s_off[kMaxXRanks + 1];
    __shared__ int4 s_h[kMaxXRanks];
    load_hdrs(xb, nr, s_h);
    const long long n = 4 * rank_prefix(ctl, s_h, nr, s_off, xb.cap, false);
    for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x) {
        const EvRec* r = rank_ev(xb, s_off, nr, e >> 2);
        const int role = (int)(e & 3);
        const int node = r->n[role];
        if (g2l[node] < 0) continue;
        const int slot = toff[tpos[node]] + atomicSub(&cnt[node], 1) - 1;  // leaves cnt zeroed
        double* o = terms + 3 * (long long)slot;
        if (role == 0) {  // c_force3[i] += f
            o[0] = r->f[0];
            o[1] = r->f[1];
            o[2] = r->f[2];
        } else {  // triangle nodes: += -f / 3.0
            o[0] = -r->f[0] / 3.0;
            o[1] = -r->f[1] / 3.0;
            o[2] = -r->f[2] / 3.0;
        }
    }
}

// deletions of this rank since the last pack -> its block (global element, step); full: every local
// deletion step (after a state reset / upload / overflow); the header carries the rank's last
// deletion step
// (count of this block: zeroed by the pack of the other parity, which also zeroes the other
// block's for the next pack -- every rank has read that one by now; a step without a deletion
// packs nothing)
__global__ void k_xr_dpack(const int* del_step, const int* del_any, int nEloc, long long E0, int* last_del, char* blk,
                           char* other, long long cap, int full, int t) {
    int* h = reinterpret_cast<int*>(blk);
    int* pl = reinterpret_cast<int*>(blk + kXHdr);
    if (blockIdx.x == 0 && threadIdx.x == 0) reinterpret_cast<int*>(other)[0] = 0;
    const bool none = !full && *del_any != t;  // block-uniform
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; !none && e < nEloc; e += gridDim.x * blockDim.x) {
        const int d = del_step[e];
        if (full) {
            pl[e] = d;
        } else if (d != last_del[e]) {
            const int k = atomicAdd(&h[0], 1);
            if (k < cap) {
                pl[2 * k] = (int)(E0 + e);
                pl[2 * k + 1] = d;
            }
        }
        last_del[e] = d;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        h[2] = *del_any;
        h[3] = full;
    }
}

// every rank's deletion block -> the global deletion steps; block 0 also the global last deletion
// step and the overflow check (a list beyond its capacity poisons the step; it is packed again,
// full, for the retry)
// The incremental blocks also hold exactly the elements deleted in the previous step: they go to
// the deletion list of the live-list update (k_ct_find_del's job on one GPU), and block 0 sets the
// update flag (after k_ct_reset, which clears the list). A full block comes with a full rebuild
// of the live lists on every rank (state reset, upload, overflow retry), which needs no list.
__global__ void k_xr_dunpack(XBlk xb, int nr, const long long* e_off, int* g_del, long long nE_g,
                             int* poison, int t, int* xctl, int* hc, unsigned int* ctl, int* dlist) {
    const int q = (int)blockIdx.y;
    const char* b = xb.p[q];
    const int* pl = reinterpret_cast<const int*>(b + kXHdr);
    __shared__ int4 s_h[kMaxXRanks];
    load_hdrs(xb, nr, s_h);
    x_counts(s_h, nr, 0, xctl, hc);
    if (s_h[q].w) {
        const long long e0 = e_off[q], ne = e_off[q + 1] - e0;
        for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < ne; k += (long long)gridDim.x * blockDim.x)
            g_del[e0 + k] = pl[k];
    } else {
        const long long n = min(s_h[q].x, xb.cap[q]);
        for (long long k = blockIdx.x * (long long)blockDim.x + threadIdx.x; k < n;
             k += (long long)gridDim.x * blockDim.x) {
            const int e = pl[2 * k], d = pl[2 * k + 1];
            g_del[e] = d;
            if (d == t - 1) dlist[atomicAdd(&ctl[kNdel], 1u)] = e;
        }
    }
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
        int mx = 0;
        bool over = false;
        for (int r = 0; r < nr; ++r) {
            mx = max(mx, s_h[r].z);
            over |= !s_h[r].w && s_h[r].x > xb.cap[r];
        }
        g_del[nE_g + 1] = mx;
        ctl[kDel] = (ctl[kDirty] == 0 && mx == t - 1) ? 1u : 0u;
        const int pstep = t;
        if (over) {
            atomicOr(xctl, 1);
            if (poison[0] == 0) {
                poison[1] = pstep;
                poison[0] = 1;
            }
        }
    }
}

// A1 of a step without a full rebuild (multi-GPU), ONE 1024-thread workgroup: k_ct_reset's share of
// the phase (event and candidate counters, this step's partial box words and bin block header, the
// bucket-head sequence), and every rank's deletion records into the global deletion steps and the
// deletion list; k_ct_append follows with a full grid (in this workgroup, a wave per deleted
// element, the append took 35-63 µs on C4's deletion steps against 15-18 µs for the grid). A rank's
// block that is full (a peer out of step) is unpacked too. The previous step's touched forces and the term counter are
// phase B's (k_ct_count_g), the touched counter the previous k_ct_sum's.
__global__ __launch_bounds__(1024) void k_xr_front(XBlk xb, int nr, const long long* e_off, int* g_del,
                                                   long long nE_g, int* poison, int t, int* xctl, int* hc,
                                                   unsigned int* ctl, int* dlist, unsigned long long* bbox,
                                                   int npairs, unsigned int* evs, unsigned int* ccnt, int* zero_hdr) {
    __shared__ int4 s_h[kMaxXRanks];
    load_hdrs(xb, nr, s_h);
    x_counts(s_h, nr, 0, xctl, hc);
    const int tid = (int)threadIdx.x, bd = (int)blockDim.x;
    if (tid < kEvShards) evs[tid * kShardStride] = 0;
    if (tid < kCandShards)
        ccnt[tid * kShardStride] = ccnt[tid * kShardStride + kTestWord] = ccnt[tid * kShardStride + kItemWord] = 0;
    for (int q = tid; q < box_words(npairs); q += bd) bbox[q] = box_max(q) ? 0ULL : ~0ULL;
    if (tid < 2) zero_hdr[tid] = 0;
    if (tid == 0) {
        int mx = 0;
        bool over = false;
        for (int r = 0; r < nr; ++r) {
            mx = max(mx, s_h[r].z);
            over |= !s_h[r].w && s_h[r].x > xb.cap[r];
        }
        g_del[nE_g + 1] = mx;
        ctl[kEv] = 0;
        ctl[kDirty] = 0;
        ctl[kNdel] = 0;
        ctl[kNcand] = 0;
        ctl[kCandOver] = 0;
        ctl[kSeq] = ctl[kSeq] + 1u;
        ctl[kDel] = mx == t - 1 ? 1u : 0u;
        if (over) {
            atomicOr(xctl, 1);
            if (poison[0] == 0) {
                poison[1] = t;
                poison[0] = 1;
            }
        }
        __threadfence();  // (the counters before the other waves' atomics and agent-scope loads)
    }
    __syncthreads();
    for (int q = 0; q < nr; ++q) {
        const int* pl = reinterpret_cast<const int*>(xb.p[q] + kXHdr);
        if (s_h[q].w) {
            const long long e0 = e_off[q], ne = e_off[q + 1] - e0;
            for (long long k = tid; k < ne; k += bd) g_del[e0 + k] = pl[k];
        } else {
            const long long n = min(s_h[q].x, xb.cap[q]);
            for (long long k = tid; k < n; k += bd) {
                const int e = pl[2 * k], d = pl[2 * k + 1];
                g_del[e] = d;
                if (d == t - 1) dlist[atomicAdd(&ctl[kNdel], 1u)] = e;
            }
        }
    }
}

// pair boxes of all ranks: min of the min words, max of the max words (exact, order-free). RCCL
// all-reduces with MIN: the max words travel complemented (k_xr_boxflip before and after).
__global__ void k_xr_boxflip(unsigned long long* bb, int npairs) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q < box_words(npairs) && box_max(q)) bb[q] = ~bb[q];
}
struct XBox {
    const unsigned long long* p[kMaxXRanks];
};
__global__ void k_xr_boxcomb(XBox xb, int nr, int npairs, unsigned long long* out) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= box_words(npairs)) return;
    const bool mx = box_max(q);
    unsigned long long v = xb.p[0][q];
    for (int r = 1; r < nr; ++r) {
        const unsigned long long w = xb.p[r][q];
        v = mx ? umax64(v, w) : umin64(v, w);
    }
    out[q] = v;
}

// A2: the pair boxes of every rank combined (each workgroup in LDS; workgroup 0 also stores them
// for the triangle prefilter of A3), then this rank's live i-nodes inside their pair's range box ->
// compact records in its block. xb: the in-process peers' partial boxes (nxb = nranks), or the
// RCCL all-reduced one (nxb = 1, max words complemented: flip). npairs > kLdsPairs: k_xr_boxcomb
// combined them into boxg before (nxb = 0).
constexpr int kLdsPairs = 64;
__global__ __launch_bounds__(kB) void k_xr_bin(StepIn s, const Seg* segs, int nseg, const int* reg,
                                               const int* ni_live, const int* ni_pair, const int* ni_node,
                                               const PairParam* par, XBox xb, int nxb, int flip, int npairs,
                                               unsigned long long* boxg, char* blk, long long cap, int sb) {
#pragma clang fp contract(off)
    __shared__ unsigned s_app[2];
    __shared__ alignas(16) unsigned long long s_bb[12 * kLdsPairs + 1];
    const unsigned long long* bbox = boxg;
    if (nxb > 0) {
        for (int q = (int)threadIdx.x; q < box_words(npairs); q += kB) {
            const bool mx = box_max(q);
            unsigned long long v = xb.p[0][q];
            for (int r = 1; r < nxb; ++r) {
                const unsigned long long w = xb.p[r][q];
                v = mx ? umax64(v, w) : umin64(v, w);
            }
            if (flip && mx) v = ~v;
            s_bb[q] = v;
            if (blockIdx.x == 0) boxg[q] = v;
        }
        __syncthreads();
        bbox = s_bb;
    }
    if ((int)blockIdx.x / sb >= nseg) return;  // (nseg = 0: one workgroup, the boxes only)
    const Seg sg = segs[blockIdx.x / sb];
    if (sg.side != 0) return;  // block-uniform
    const int base = reg[2 * sg.region], n = reg[2 * sg.region + 1];
    unsigned int* cnt = reinterpret_cast<unsigned int*>(blk);
    BRec* out = reinterpret_cast<BRec*>(blk + kXHdr);
    for (int q0 = (blockIdx.x % sb) * kB; q0 < n; q0 += sb * kB) {  // block-uniform trip count
        const int q = q0 + (int)threadIdx.x;
        bool in = false;
        int nd = 0, pr = 0;
        double p[3] = {0.0, 0.0, 0.0};
        Range r;
        r.empty = true;
        if (q < n) {
            const int k = ni_live[base + q];
            pr = ni_pair[k];
            r = pair_range(bbox + 12 * pr);
            nd = ni_node[k];
            pos(s, nd, p);
            in = !(r.empty || p[0] < r.mn[0] || p[1] < r.mn[1] || p[2] < r.mn[2] || p[0] > r.mx[0] ||
                   p[1] > r.mx[1] || p[2] > r.mx[2]);  // the candidate test of :2514-2519
        }
        const unsigned slot = block_append(cnt, in, s_app);
        if (in && (long long)slot < cap) {
            BRec e;
            bin_rec(s, r, par[pr], pr, nd, p, e);
            out[slot] = e;
        }
    }
}

// A3: every gathered record (rank q's record k at slot xb.off[q] + k of the bucket list) pushed onto
// its bucket's chain; xctl bit 2 and the poison when a rank binned more than its block holds
// (workgroup bx of gbx over rank q's block)
__device__ __forceinline__ void insert_body(int bx, int gbx, int q, const XBlk& xb, int nr,
                                            const PairParam* par, const unsigned int* ctl, unsigned long long* head,
                                            BEnt* blist, BVel* bvel, int* poison, int pstep, int* xctl, int* hc) {
    __shared__ int4 s_h[kMaxXRanks];
    load_hdrs(xb, nr, s_h);
    x_overflow_check(s_h, nr, xb.cap, poison, pstep, xctl, 2);
    x_counts(s_h, nr, 1, xctl, hc);
    const long long n = min(s_h[q].x, xb.cap[q]);
    const unsigned seq = ctl[kSeq];
    const uint4* rec = reinterpret_cast<const uint4*>(xb.p[q] + kXHdr);  // 6 x 16 B per record
    for (long long k = bx * (long long)blockDim.x + threadIdx.x; k < n; k += (long long)gbx * blockDim.x) {
        // the record moves as six 16-B vectors (a by-value BRec became a 96-B private array in LDS)
        uint4 w[6];
#pragma unroll
        for (int v = 0; v < 6; ++v) w[v] = rec[6 * k + v];
        const PairParam& pp = par[(int)w[1].w];  // BEnt: m[3] = w0.xy w0.zw w1.xy, node w1.z, pad w1.w
        const int b = pp.hash_off + (int)(hash3(ll2(w[0].x, w[0].y), ll2(w[0].z, w[0].w), ll2(w[1].x, w[1].y)) &
                                          (unsigned)(pp.hash_size - 1));
        const int slot = xb.off[q] + (int)k;
        const unsigned long long old = atomicExch(&head[b], ((unsigned long long)seq << 32) | (unsigned)slot);
        const long long nx = (unsigned)(old >> 32) == seq ? (long long)(unsigned)old : -1LL;
        w[3].z = (unsigned)(unsigned long long)nx;  // BEnt::next, the last 8 B
        w[3].w = (unsigned)((unsigned long long)nx >> 32);
        uint4* be = reinterpret_cast<uint4*>(blist + slot);
        uint4* bv = reinterpret_cast<uint4*>(bvel + slot);
#pragma unroll
        for (int v = 0; v < 4; ++v) be[v] = w[v];
        bv[0] = w[4];
        bv[1] = w[5];
    }
}

__global__ void k_xr_insert(XBlk xb, int nr, const PairParam* par, const unsigned int* ctl,
                            unsigned long long* head, BEnt* blist, BVel* bvel, int* poison, int pstep, int* xctl,
                            int* hc) {
    insert_body(blockIdx.x, gridDim.x, blockIdx.y, xb, nr, par, ctl, head, blist, bvel, poison, pstep, xctl, hc);
}

// A3 with the triangle prefilter in the same launch (workgroups [0, gb * nr) insert, the rest
// filter: independent work, side by side)
__global__ __launch_bounds__(kB) void k_xr_insfilter(XBlk xb, int nr, const PairParam* par,
                                                     const unsigned int* ctl, unsigned long long* head, BEnt* blist,
                                                     BVel* bvel, int* poison, int pstep, int* xctl, int* hc, int gb,
                                                     StepIn s, const int* tri_cnt, const int* tri_live,
                                                     const int* tri_pair, const int* tri_nodes, const int* tri_ele,
                                                     const unsigned long long* bbox, unsigned int* ccnt, TriRec* cand,
                                                     long long cshard_cap, uint2* item) {
    const int ni = gb * nr;
    if ((int)blockIdx.x < ni)
        insert_body(blockIdx.x % gb, gb, blockIdx.x / gb, xb, nr, par, ctl, head, blist, bvel, poison, pstep,
                    xctl, hc);
    else
        tri_filter_body(blockIdx.x - ni, gridDim.x - ni, s, tri_cnt, tri_live, tri_pair, tri_nodes, tri_ele, par, bbox,
                        ccnt, cand, cshard_cap, item);
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
template <class T>
hipError_t upload(T** p, const std::vector<T>& v, hipStream_t s) {
    hipError_t e = dalloc(p, v.size());
    if (e != hipSuccess || v.empty()) return e;
    return hipMemcpyAsync(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
}

// ---- host: surface extraction with the reference's semantics ------------------------------
struct Face {
    int n[4];    // oriented (global 0-based nodes)
    int key[4];  // sorted
    int ele;     // global 0-based element
};

struct Inst {
    int e0 = -1, nE = 0;
    std::vector<Face> faces;       // 6 per element, in the reference's order
    std::vector<int> order;        // face indices sorted by (key, index)
    std::vector<int> exterior;     // exterior face indices, ascending
    std::vector<std::vector<int>> added;  // per local element: faces exposed by its deletion
    double young = 0;
};

bool key_less(const Face& a, const Face& b) {
    for (int q = 0; q < 4; ++q)
        if (a.key[q] != b.key[q]) return a.key[q] < b.key[q];
    return false;
}
bool key_eq(const Face& a, const Face& b) {
    return a.key[0] == b.key[0] && a.key[1] == b.key[1] && a.key[2] == b.key[2] && a.key[3] == b.key[3];
}

void build_instance(Inst& I, const std::vector<double>& X, const std::vector<int>& conn) {
#pragma clang fp contract(off)
    static const int fidx[6][4] = {{0, 1, 2, 3}, {4, 5, 6, 7}, {0, 1, 5, 4}, {1, 2, 6, 5}, {2, 3, 7, 6}, {3, 0, 4, 7}};
    const int F = 6 * I.nE;
    I.faces.resize(F);
    for (int j = 0; j < I.nE; ++j) {  // get_element_face, :1944-1992
        const int e = I.e0 + j;
        const int* el = &conn[8 * (size_t)e];
        double ctr[3] = {0, 0, 0};
        for (int a = 0; a < 8; ++a)
            for (int c = 0; c < 3; ++c) ctr[c] += X[3 * (size_t)el[a] + c];
        for (int c = 0; c < 3; ++c) ctr[c] /= 8;
        for (int k = 0; k < 6; ++k) {
            Face& f = I.faces[6 * j + k];
            for (int q = 0; q < 4; ++q) f.n[q] = el[fidx[k][q]];
            const double* x1 = &X[3 * (size_t)f.n[0]];
            const double* x2 = &X[3 * (size_t)f.n[1]];
            const double* x4 = &X[3 * (size_t)f.n[3]];
            const double v1[3] = {x2[0] - x1[0], x2[1] - x1[1], x2[2] - x1[2]};
            const double v2[3] = {x4[0] - x1[0], x4[1] - x1[1], x4[2] - x1[2]};
            const double nv[3] = {v1[1] * v2[2] - v1[2] * v2[1], v1[2] * v2[0] - v1[0] * v2[2],
                                  v1[0] * v2[1] - v1[1] * v2[0]};
            const double vc[3] = {ctr[0] - x1[0], ctr[1] - x1[1], ctr[2] - x1[2]};
            if (nv[0] * vc[0] + nv[1] * vc[1] + nv[2] * vc[2] > 0.) std::swap(f.n[1], f.n[3]);
            for (int q = 0; q < 4; ++q) f.key[q] = f.n[q];
            std::sort(f.key, f.key + 4);
            f.ele = e;
        }
    }
    // faces ordered by (key, index): counting sort on the smallest node, then a stable insertion
    // sort inside each (tiny) bucket -- linear time at millions of faces
    I.order.resize(F);
    {
        int kmin = INT32_MAX, kmax = -1;
        for (const Face& f : I.faces) {
            kmin = std::min(kmin, f.key[0]);
            kmax = std::max(kmax, f.key[0]);
        }
        const int nb = F ? kmax - kmin + 1 : 0;
        std::vector<int> start((size_t)nb + 1, 0);
        for (const Face& f : I.faces) start[f.key[0] - kmin + 1]++;
        for (int b = 0; b < nb; ++b) start[b + 1] += start[b];
        std::vector<int> fill(start.begin(), start.end() - 1);
        for (int i = 0; i < F; ++i) I.order[fill[I.faces[i].key[0] - kmin]++] = i;  // ascending index per bucket
        for (int b = 0; b < nb; ++b)
            for (int q = start[b] + 1; q < start[b + 1]; ++q) {
                const int v = I.order[q];
                int r = q - 1;
                while (r >= start[b] && key_less(I.faces[v], I.faces[I.order[r]])) {
                    I.order[r + 1] = I.order[r];
                    --r;
                }
                I.order[r + 1] = v;
            }
    }
    // get_surface_triangle's scan (:2040-2084): in each run of equal keys o1<o2<..<om the scan
    // pairs (o1,o2), (o3,o4), ...; an odd run keeps its LAST face, unless that is the very last
    // face of the instance (the loop stops at nE*6-1) -- SURVEY §9 Q13.
    I.exterior.clear();
    for (int a = 0; a < F;) {
        int b = a;
        while (b < F && key_eq(I.faces[I.order[a]], I.faces[I.order[b]])) ++b;
        const int m = b - a;
        const int last = I.order[b - 1];
        if ((m & 1) && last != F - 1) I.exterior.push_back(last);
        a = b;
    }
    std::sort(I.exterior.begin(), I.exterior.end());
    // add_surface_triangle (:2167-2245): for each face of the deleted element, the FIRST face (in
    // face order) with the same key that belongs to another element
    I.added.assign(I.nE, {});
    std::vector<int> run_start(F), pos_in_order(F);
    for (int i = 0; i < F; ++i) pos_in_order[I.order[i]] = i;
    for (int a = 0; a < F;) {
        int b = a;
        while (b < F && key_eq(I.faces[I.order[a]], I.faces[I.order[b]])) ++b;
        for (int q = a; q < b; ++q) run_start[I.order[q]] = a;
        a = b;
    }
    for (int j = 0; j < I.nE; ++j)
        for (int k = 0; k < 6; ++k) {
            const int fi = 6 * j + k;
            for (int q = run_start[fi]; q < F && key_eq(I.faces[I.order[q]], I.faces[fi]); ++q) {
                const int cand = I.order[q];
                if (I.faces[cand].ele == I.e0 + j) continue;
                I.added[j].push_back(cand);
                break;
            }
        }
}

}  // namespace

namespace hkc {

void contact_destroy(hakai_ctx* c) {
    Contact* C = c->contact;
    if (!C) return;
    (void)hipStreamSynchronize(c->stream);
    dfree(C->d_par);
    dfree(C->d_seg);
    dfree(C->d_ni_pair); dfree(C->d_ni_node); dfree(C->d_ni_orig); dfree(C->d_ni_aptr); dfree(C->d_ni_add);
    dfree(C->d_nj_pair); dfree(C->d_nj_node); dfree(C->d_nj_orig); dfree(C->d_nj_aptr); dfree(C->d_nj_add);
    dfree(C->d_tri_pair); dfree(C->d_tri_nodes); dfree(C->d_tri_ele); dfree(C->d_tri_adder);
    if (C->d_tiles) (void)hipFree(C->d_tiles);
    dfree(C->d_tile_cnt); dfree(C->d_tile_off); dfree(C->d_reg_first); dfree(C->d_reg); dfree(C->d_pair_reg);
    dfree(C->d_el_tri_ptr); dfree(C->d_el_tri); dfree(C->d_el_ni_ptr); dfree(C->d_el_ni); dfree(C->d_el_nj_ptr);
    dfree(C->d_el_nj); dfree(C->d_dlist);
    dfree(C->d_ni_live); dfree(C->d_nj_live); dfree(C->d_tri_live);
    dfree(C->d_head); dfree(C->d_blist); dfree(C->d_bvel);
    dfree(C->d_bbox); dfree(C->d_ctl); dfree(C->d_evs); dfree(C->d_ev_nodes); dfree(C->d_ev_f); dfree(C->d_cnt); dfree(C->d_tpos);
    dfree(C->d_touched[0]); dfree(C->d_touched[1]); dfree(C->d_toff); dfree(C->d_tcnt); if (C->d_cand) (void)hipFree(C->d_cand);
    dfree(C->d_terms); dfree(C->d_velo0); dfree(C->d_ccnt); dfree(C->d_item);
    if (Xrank* X = C->xr) {
        (void)hipDeviceSynchronize();  // in-process peers may still read this rank's blocks
        dfree(X->d_l2g); dfree(X->d_g2l); dfree(X->g_mass); dfree(X->g_del); dfree(X->d_last_del);
        for (int x = 0; x < Xrank::kNx; ++x) {
            dfree(X->d_send[x][0]);
            dfree(X->d_send[x][1]);
            dfree(X->d_recv[x]);
            for (auto& e : X->ev_sent[x])
                if (e) (void)hipEventDestroy(e);
        }
        dfree(X->d_box[0]); dfree(X->d_box[1]); dfree(X->d_boxg); dfree(X->d_xctl);
        for (auto& e : X->ev_box)
            if (e) (void)hipEventDestroy(e);
        for (auto& e : X->ev_cnt)
            if (e) (void)hipEventDestroy(e);
        if (X->h_cnt) (void)hipHostFree(X->h_cnt);
        delete X;
    }
    delete C;
    c->contact = nullptr;
    dfree(c->d_fext);
}

// ---- multi-GPU exchange (Xrank) ------------------------------------------------------------------
static size_t xr_rec_bytes(int x) { return x == 0 ? 8 : (x == 1 ? sizeof(BRec) : sizeof(EvRec)); }
// block bytes of rank q's block of exchange x at its capacity (deletions, full: room for every local
// deletion step of the largest rank)
static size_t xr_blkq(const Xrank* X, int x, int q, bool full = false) {
    size_t b = kXHdr + xr_rec_bytes(x) * (size_t)X->capq[x][q];
    if (x == 0 && full) b = kXHdr + 4 * (size_t)X->maxEloc;
    return (b + 15) / 16 * 16;
}
static size_t xr_alloc_blk(const Xrank* X, int x, int q) {
    return x == 0 ? std::max(xr_blkq(X, 0, q, false), xr_blkq(X, 0, q, true)) : xr_blkq(X, x, q);
}
// every rank's block bytes and their offsets in the receive buffer
static size_t xr_layout(const Xrank* X, int x, bool full, size_t* bytes, size_t* off) {
    size_t run = 0;
    for (int q = 0; q < X->nranks; ++q) {
        bytes[q] = xr_blkq(X, x, q, full);
        off[q] = run;
        run += bytes[q];
    }
    return run;
}
// records of the largest block / of all blocks of exchange x
static void xr_cap_sums(Xrank* X, int x) {
    long long mx = 0;
    for (long long v : X->capq[x]) mx = std::max(mx, v);
    X->cap[x] = mx;
}
static long long xr_cap_total(const Xrank* X, int x) {
    long long t = 0;
    for (long long v : X->capq[x]) t += v;
    return t;
}

// send (both parities) and receive buffers for the current capacities; bucket-record and
// bucket-list arrays for the binned records of all ranks. Capacities may shrink (xr_grow); a
// buffer is reallocated only when a capacity outgrows it, then with 1.25x room (a reallocation
// synchronises the device).
static int xr_buffers(hakai_ctx* c) {
    Contact* C = c->contact;
    Xrank* X = C->xr;
    const int nr = X->nranks, me = X->rank;
    bool sync = false;
    size_t need_send[Xrank::kNx], need_recv[Xrank::kNx];
    for (int x = 0; x < Xrank::kNx; ++x) {
        need_send[x] = xr_alloc_blk(X, x, me);
        need_recv[x] = 0;
        for (int q = 0; q < nr; ++q) need_recv[x] += xr_alloc_blk(X, x, q);
        sync |= X->send_bytes[x] < need_send[x] || (comm_is_rccl(c) && X->recv_bytes[x] < need_recv[x]);
    }
    const long long nb = xr_cap_total(X, 1);
    sync |= C->blist_cap < nb;
    if (!sync) return 0;
    HIPCHK(hipDeviceSynchronize());  // (in-process peers read the send blocks)
    auto room = [](size_t b) { return (b + b / 4 + 15) / 16 * 16; };
    for (int x = 0; x < Xrank::kNx; ++x) {
        if (X->send_bytes[x] < need_send[x]) {
            const size_t b = room(need_send[x]);
            for (int p = 0; p < 2; ++p) {
                dfree(X->d_send[x][p]);
                HIPCHK(dalloc(&X->d_send[x][p], b));
                HIPCHK(hipMemset(X->d_send[x][p], 0, b));
            }
            X->send_bytes[x] = b;
        }
        if (comm_is_rccl(c) && X->recv_bytes[x] < need_recv[x]) {
            const size_t b = room(need_recv[x]);
            dfree(X->d_recv[x]);
            HIPCHK(dalloc(&X->d_recv[x], b));
            X->recv_bytes[x] = b;
        }
    }
    if (C->blist_cap < nb) {
        const long long n = nb + nb / 4;
        dfree(C->d_blist);
        dfree(C->d_bvel);
        HIPCHK(dalloc(&C->d_blist, (size_t)n));
        HIPCHK(dalloc(&C->d_bvel, (size_t)n));
        C->blist_cap = n;
    }
    return 0;
}

// the blocks of exchange x, parity par, of every rank: gathered over RCCL into the receive buffer
// (one grouped send/receive per peer, each block at its own rank's size), or read in place from the
// in-process peers (after a stream wait on their "sent" event); with every block's capacity and
// slot offset
static int xr_gather(hakai_ctx* c, int x, int par, bool full, XBlk& xb) {
    Xrank* X = c->contact->xr;
    const int nr = X->nranks;
    if (nr > kMaxXRanks) return fail(HAKAI_ERR_COMM, "multi-GPU contact: more than %d ranks", kMaxXRanks);
    long long run = 0;
    for (int q = 0; q < nr; ++q) {
        xb.cap[q] = (int)X->capq[x][q];
        xb.off[q] = (int)run;
        run += X->capq[x][q];
    }
    if (run > (long long)INT_MAX)  // (record slots and bucket-list indices are 32-bit)
        return fail(HAKAI_ERR_STATE, "multi-GPU contact: %lld exchange records over the ranks exceed 2^31", run);
    if (comm_is_rccl(c)) {
        size_t bytes[kMaxXRanks], off[kMaxXRanks];
        xr_layout(X, x, full, bytes, off);
        if (int rc = comm_allgatherv_raw(c, X->d_send[x][par], X->d_recv[x], bytes, off)) return rc;
        for (int q = 0; q < nr; ++q) xb.p[q] = q == X->rank ? X->d_send[x][par] : X->d_recv[x] + off[q];
        return 0;
    }
    for (int q = 0; q < nr; ++q) {
        hakai_ctx* pc = comm_peer_ctx(c, q);
        Xrank* P = pc && pc->contact ? pc->contact->xr : nullptr;
        // the peer packed this step's block: deletions at the end of the previous step (seq), bins in
        // this step's A2 (same seq and step), events in this step's A3 (same A3 count; a peer may have
        // ended the step already)
        const bool same = P && P->capq[x] == X->capq[x] &&
                          (x == 0 ? P->seq == X->seq
                                  : x == 1 ? P->seq == X->seq && P->t_a == X->t_a : P->phase_a == X->phase_a);
        if (!same)
            return fail(HAKAI_ERR_STATE, "multi-GPU contact: rank %d is not at the same step (step an in-process group "
                        "with hakai_step_group; hakai_set_contact_global, reset and upload on every rank)", q);
        if (q != X->rank) HIPCHK(hipStreamWaitEvent(c->stream, P->ev_sent[x][par], 0));
        xb.p[q] = P->d_send[x][par];
    }
    return 0;
}

// this rank's deletions since the last pack (or, full, every local deletion step) -> the deletion
// block of step X->seq
static int xr_dpack(hakai_ctx* c, bool full) {
    Xrank* X = c->contact->xr;
    const int par = (int)(X->seq & 1);
    if (full) HIPCHK(hipMemsetAsync(X->d_send[0][par], 0, kXHdr, c->stream));
    const int n = (int)std::max<long long>(X->nEloc, 1);
    hipLaunchKernelGGL(k_xr_dpack, dim3((unsigned)std::min((n + kB - 1) / kB, 1024)), dim3(kB), 0, c->stream,
                       c->d_del_step, c->d_del_step + c->nEp + 1, (int)X->nEloc, X->E0, X->d_last_del,
                       X->d_send[0][par], X->d_send[0][1 - par], X->capq[0][X->rank], full ? 1 : 0, X->t_a);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(X->ev_sent[0][par], c->stream));
    X->full_del = full;
    return 0;
}

// Capacity of a block from its rank's recent counts: 1.25x the largest of the last kHist gathered
// counts plus a floor of records (the counts are two steps old when read: a burst beyond the
// headroom overflows, and the step runs again with the capacity grown past it, contact_after_overflow).
// Deletion blocks (8 B records, bursts at deletion waves) keep a floor of 1024 records.
static long long xr_cap_target(const Xrank* X, int x, long long mx) {
    return std::min<long long>(X->cap_max[x], std::max<long long>(X->cap_floor[x], mx + mx / 4 + (mx > 0 ? 32 : 0)));
}
// Capacities from the counts gathered two steps ago (the same numbers on every rank, so every rank
// sizes every block alike): a rank's block grows to its target at once and shrinks to it once it
// exceeds 1.5x the target (the headroom window keeps a recent burst's size). Exchange x in [x0, x1):
// the deletion block changes before it is packed (end of a step), the bin and event blocks at the
// start of the step that packs them -- never while an in-process peer may still read the block of
// the step before.
static int xr_grow(hakai_ctx* c, int x0, int x1) {
    Xrank* X = c->contact->xr;
    if (X->cnt_seq < 2) return 0;
    const long long sl = (X->cnt_seq - 2) & 3;
    HIPCHK(hipEventSynchronize(X->ev_cnt[sl]));
    const int* h = X->h_cnt + (size_t)sl * Xrank::kNx * X->nranks;
    const int nr = X->nranks, H = Xrank::kHist;
    for (int x = x0; x < x1; ++x) {
        for (int q = 0; q < nr; ++q) {
            int* hq = X->hist[x].data() + (size_t)q * H;
            hq[(X->cnt_seq - 2) % H] = h[x * nr + q];
            long long mx = 0;
            for (int j = 0; j < H; ++j) mx = std::max<long long>(mx, hq[j]);
            const long long tg = xr_cap_target(X, x, mx);
            long long& cq = X->capq[x][q];
            if (tg > cq || 2 * cq > 3 * tg) cq = tg;
        }
        xr_cap_sums(X, x);
    }
    return xr_buffers(c);
}

int contact_state_reset(hakai_ctx* c, const double* velo0_host) {
    Contact* C = c->contact;
    if (!C) return 0;
    C->use_velo0 = true;
    C->force_rebuild = true;
    if (velo0_host)
        HIPCHK(hipMemcpyAsync(C->d_velo0, velo0_host, 3 * (size_t)c->nN * sizeof(double), hipMemcpyHostToDevice,
                              c->stream));
    if (Xrank* X = C->xr) {  // every deletion step travels with the next block
        HIPCHK(hipMemsetAsync(X->g_del, 0, ((size_t)X->nE_g + 2) * sizeof(int), c->stream));
        HIPCHK(hipMemsetAsync(X->d_xctl, 0, (4 + 2 * (size_t)Xrank::kNx * X->nranks) * sizeof(int), c->stream));
        X->seq = 0;
        X->cnt_seq = 0;
        return xr_dpack(c, true);
    }
    return 0;
}

// multi-GPU, after the element kernel of a step: capacities for the next step, then this step's
// deletions into the next step's deletion block
int contact_post_step(hakai_ctx* c) {
    Contact* C = c->contact;
    if (!C || !C->xr) return 0;
    Xrank* X = C->xr;
    ++X->seq;
    if (int rc = xr_grow(c, 0, 1)) return rc;
    return xr_dpack(c, false);
}

static int search(hakai_ctx* c, const StepIn& in, bool fused);
static void tri_search(hakai_ctx* c, const StepIn& in);

// prefilter grid: one live triangle per thread
static unsigned filter_grid(const Contact* C) {
    return (unsigned)std::max(1, std::min((C->n_tri + kB - 1) / kB, kFilterBlocks));
}

// the triangle prefilter against the (combined) pair boxes bbox, as its own launch
static void tri_prefilter(hakai_ctx* c, const StepIn& in, const unsigned long long* bbox) {
    Contact* C = c->contact;
    hipLaunchKernelGGL(k_ct_tri_filter, dim3(filter_grid(C)), dim3(kB), 0, c->stream, in, C->d_reg + 2 * C->tri_reg + 1,
                       C->d_tri_live, C->d_tri_pair, C->d_tri_nodes, C->d_tri_ele, C->d_par, bbox, C->d_ccnt,
                       (TriRec*)C->d_cand, C->cshard_cap, C->small ? nullptr : C->d_item);
}

static StepIn step_in(hakai_ctx* c, double t, double d_time) {
    Contact* C = c->contact;
    StepIn in;
    in.coord = c->d_coord;
    in.u = c->d_u[c->cur];
    in.u_pre = c->d_u[1 - c->cur];
    in.flag = c->d_flag;
    in.conn = c->d_conn;
    in.mass = C->xr ? C->xr->g_mass : c->d_mass;
    in.l2g = C->xr ? C->xr->d_l2g : nullptr;
    in.del_step = C->xr ? C->xr->g_del : c->d_del_step;
    in.velo0 = C->use_velo0 ? C->d_velo0 : nullptr;
    in.d_time = d_time;
    in.t = (int)t;
    return in;
}

// Start of a step's contact work (:500-560): multi-GPU deletions of the previous step, step
// prologue, live-list update, pair boxes (a rank's partial boxes). One GPU: the whole search too.
static int step_start(hakai_ctx* c, double t, double d_time) {
    Contact* C = c->contact;
    Xrank* X = C->xr;
    hipStream_t s = c->stream;
    StepIn in = step_in(c, t, d_time);
    int* del_step = c->d_del_step;
    const int* del_any = c->d_del_step + c->nEp + 1;
    double* fext = c->d_fext;
    unsigned long long* bbox = C->d_bbox;
    XBlk xb{};
    if (X) {
        if (int rc = xr_grow(c, 1, Xrank::kNx)) return rc;
        X->t_a = in.t;
        X->par_a = (int)(X->seq & 1);
        X->sl_a = (int)(X->cnt_seq & 3);
        if (int rc = xr_gather(c, 0, X->par_a, X->full_del, xb)) return rc;
        del_step = X->g_del;
        del_any = X->g_del + X->nE_g + 1;
        bbox = X->d_box[X->par_a];
    }
    if ((long long)in.t != C->last_t + 1 || C->always_rebuild) C->force_rebuild = true;
    const bool rebuild = C->force_rebuild;
    const int tsel = C->tsel = 1 - C->tsel;
    // small decks: reset + deletion scan + surface append in one workgroup (not on full-rebuild
    // steps, whose live-list rebuild sits between the reset and the scan)
    const bool fused = C->small && C->fuse_small && !X;
    AppendIn A;
    A.el_tri_ptr = C->d_el_tri_ptr; A.el_tri = C->d_el_tri;
    A.el_ni_ptr = C->d_el_ni_ptr; A.el_ni = C->d_el_ni; A.el_nj_ptr = C->d_el_nj_ptr; A.el_nj = C->d_el_nj;
    A.ni_orig = C->d_ni_orig; A.ni_aptr = C->d_ni_aptr; A.ni_add = C->d_ni_add; A.ni_pair = C->d_ni_pair;
    A.nj_orig = C->d_nj_orig; A.nj_aptr = C->d_nj_aptr; A.nj_add = C->d_nj_add; A.nj_pair = C->d_nj_pair;
    A.pair_reg = C->d_pair_reg;
    A.tri_reg = C->tri_reg;
    if (fused && !rebuild) {
        hipLaunchKernelGGL(k_ct_prologue1, dim3(1), dim3(kSmallThreads), 0, s, bbox, C->npairs, C->d_ctl, C->d_evs,
                           C->d_ccnt, del_any, in.t, c->g_trd, C->d_touched[1 - tsel], tsel, fext, del_step,
                           (int)C->nE, C->d_dlist, A, C->d_reg, C->d_ni_live, C->d_nj_live, C->d_tri_live,
                           C->ntile > 0 ? 1 : 0);
    } else if (X && !rebuild) {
        // multi-GPU: the reset's share and every rank's deletions in one workgroup, then the append
        hipLaunchKernelGGL(k_xr_front, dim3(1), dim3(1024), 0, s, xb, X->nranks, X->d_eoff, X->g_del,
                           X->nE_g, c->d_poison, in.t, X->d_xctl, X->d_hcnt + (size_t)X->sl_a * Xrank::kNx * X->nranks,
                           C->d_ctl, C->d_dlist, bbox, C->npairs, C->d_evs, C->d_ccnt, (int*)X->d_send[1][X->par_a]);
        if (C->ntile > 0)
            hipLaunchKernelGGL(k_ct_append, dim3(256), dim3(64), 0, s, C->d_ctl, C->d_dlist, A, del_step, in.t,
                               c->g_trd, C->d_reg, C->d_ni_live, C->d_nj_live, C->d_tri_live);
    } else {
        hipLaunchKernelGGL(k_ct_reset, dim3(C->g_reset), dim3(kB), 0, s, bbox, C->npairs, C->d_ctl, C->d_evs, C->d_ccnt,
                           C->force_rebuild ? 1 : 0, X ? nullptr : del_any, in.t, c->g_trd, C->d_touched[1 - tsel], tsel,
                           fext, X ? X->d_g2l : nullptr, X ? (int*)X->d_send[1][X->par_a] : nullptr);
        if (X) {  // the deletions of every rank (after the reset: they fill its deletion list)
            const unsigned gx = (unsigned)std::min<long long>(std::max<long long>((X->maxEloc + kB - 1) / kB, 1), 256);
            hipLaunchKernelGGL(k_xr_dunpack, dim3(gx, (unsigned)X->nranks), dim3(kB), 0, s, xb, X->nranks,
                               X->d_eoff, X->g_del, X->nE_g, c->d_poison, in.t, X->d_xctl,
                               X->d_hcnt + (size_t)X->sl_a * Xrank::kNx * X->nranks, C->d_ctl, C->d_dlist);
        }
        if (C->ntile > 0) {
            LiveIn L;
            L.ni_orig = C->d_ni_orig; L.ni_aptr = C->d_ni_aptr; L.ni_add = C->d_ni_add;
            L.nj_orig = C->d_nj_orig; L.nj_aptr = C->d_nj_aptr; L.nj_add = C->d_nj_add;
            L.tri_ele = C->d_tri_ele; L.tri_adder = C->d_tri_adder;
            L.flag = in.flag; L.del_step = del_step; L.t = in.t;
            const Tile* tl = (const Tile*)C->d_tiles;
            const unsigned gt = (unsigned)std::min(C->ntile, 2048);
            // full rebuild (forced steps only: the host knows them, so the kernels are not even launched
            // otherwise)
            if (rebuild) {
                hipLaunchKernelGGL(k_ct_live_count, dim3(gt), dim3(kB), 0, s, C->d_ctl, L, tl, C->ntile, C->d_tile_cnt);
                hipLaunchKernelGGL(k_ct_live_scan, dim3(1), dim3(kB), 0, s, C->d_ctl, C->ntile, C->d_tile_cnt,
                                   C->d_tile_off, C->nreg, C->d_reg_first, C->d_reg);
                hipLaunchKernelGGL(k_ct_live_write, dim3(gt), dim3(kB), 0, s, C->d_ctl, L, tl, C->ntile, C->d_tile_off,
                                   C->d_reg_first, C->d_reg, C->d_ni_live, C->d_nj_live, C->d_tri_live);
            }
            // incremental update (steps after a deletion; multi-GPU: k_xr_dunpack listed them)
            if (!X)
                hipLaunchKernelGGL(k_ct_find_del, dim3(C->g_del), dim3(kB), 0, s, C->d_ctl, del_step, (int)C->nE, in.t,
                                   c->g_trd, C->d_dlist);
            hipLaunchKernelGGL(k_ct_append, dim3(256), dim3(64), 0, s, C->d_ctl, C->d_dlist, A, del_step, in.t,
                               c->g_trd, C->d_reg, C->d_ni_live, C->d_nj_live, C->d_tri_live);
        }
    }
    C->force_rebuild = false;
    C->last_t = in.t;
    const Seg* sg = (const Seg*)C->d_seg;
    if (C->nseg > 0)
        hipLaunchKernelGGL(k_ct_bbox, dim3(C->nseg * C->g_box), dim3(kB), 0, s, in, sg, C->d_reg, C->d_ni_live,
                           C->d_nj_live, C->d_ni_node, C->d_nj_node, bbox, C->g_box);
    HIPCHK(hipGetLastError());
    if (X) {
        HIPCHK(hipEventRecord(X->ev_box[X->par_a], s));
        return 0;
    }
    return search(c, in, fused);
}

// binning, bucket scan and fill, triangle prefilter and search, and (one GPU) the event gather
// into external_force
static int search(hakai_ctx* c, const StepIn& in, bool fused) {
    Contact* C = c->contact;
    hipStream_t s = c->stream;
    const int tsel = C->tsel;
    const unsigned gfilt = filter_grid(C);
    // the binning and the triangle prefilter in one launch (both need only the boxes; their
    // workgroups run side by side): small decks, and larger ones unless tuned off
    const bool fused_mid = (fused || C->fuse_binfilter) && C->nseg > 0 && C->n_tri > 0;
    const Seg* sg = (const Seg*)C->d_seg;
    if (C->nseg > 0) {
        if (fused_mid) {
            const int nbin = C->nseg * C->g_seg;
            hipLaunchKernelGGL(k_ct_binfilter, dim3((unsigned)nbin + gfilt), dim3(kB), 0, s, in, sg, C->d_reg,
                               C->d_ni_live, C->d_ni_pair, C->d_ni_node, C->d_par, C->d_bbox, C->d_ctl, C->d_head,
                               C->d_blist, C->d_bvel, C->g_seg, nbin, C->d_reg + 2 * C->tri_reg + 1, C->d_tri_live,
                               C->d_tri_pair, C->d_tri_nodes, C->d_tri_ele, C->d_ccnt, (TriRec*)C->d_cand,
                               C->cshard_cap, C->small ? nullptr : C->d_item);
        } else {
            hipLaunchKernelGGL(k_ct_bin, dim3(C->nseg * C->g_seg), dim3(kB), 0, s, in, sg, C->d_reg, C->d_ni_live,
                               C->d_ni_pair, C->d_ni_node, C->d_par, C->d_bbox, C->d_ctl, C->d_head, C->d_blist,
                               C->d_bvel, C->g_seg);
        }
    }
    if (C->n_tri > 0) {
        if (!fused_mid) tri_prefilter(c, in, C->d_bbox);
        tri_search(c, in);
    }
    const unsigned ge = (unsigned)C->g_ev;
    if (fused) {  // small decks: count, alloc, scatter and sum in one workgroup
        hipLaunchKernelGGL(k_ct_gather1, dim3(1), dim3(kSmallThreads), 0, s, C->d_ctl, C->d_evs, C->cap / kEvShards,
                           C->d_ev_nodes, C->d_ev_f, C->d_cnt, C->d_touched[tsel], C->d_tpos, tsel, c->d_poison,
                           in.t, c->g_trd, C->d_toff, C->d_tcnt, C->d_terms, c->d_fext);
        HIPCHK(hipGetLastError());
        C->use_velo0 = false;
        return 0;
    }
    hipLaunchKernelGGL(k_ct_count, dim3(ge), dim3(kB), 0, s, C->d_ctl, C->d_evs, C->cap / kEvShards, C->d_ev_nodes,
                       C->d_cnt, C->d_touched[tsel], C->d_tpos, tsel, c->d_poison, in.t, c->g_trd);
    hipLaunchKernelGGL(k_ct_alloc, dim3(C->g_node), dim3(kB), 0, s, C->d_ctl, tsel, C->d_touched[tsel], C->d_cnt, C->d_toff,
                       C->d_tcnt);
    hipLaunchKernelGGL(k_ct_scatter, dim3(ge), dim3(kB), 0, s, C->d_ctl, C->d_evs, C->cap / kEvShards, C->d_ev_nodes,
                       C->d_ev_f, C->d_toff, C->d_tpos, C->d_cnt, C->d_terms);
    hipLaunchKernelGGL(k_ct_sum, dim3(C->g_node), dim3(kB), 0, s, C->d_ctl, tsel, C->d_touched[tsel], C->d_toff, C->d_tcnt,
                       C->d_terms, c->d_fext, nullptr);
    HIPCHK(hipGetLastError());
    C->use_velo0 = false;
    return 0;
}

static void tri_search(hakai_ctx* c, const StepIn& in) {
    Contact* C = c->contact;
    if (C->small) {
        hipLaunchKernelGGL(k_ct_tri32, dim3(C->g_tri), dim3(128), 0, c->stream, in, C->d_ctl, C->d_ccnt,
                           (const TriRec*)C->d_cand, C->cshard_cap, C->d_par, C->d_head, C->d_blist, C->d_bvel,
                           C->d_lim, C->myu, C->d_evs, C->cap / kEvShards, C->d_ev_nodes, C->d_ev_f);
        return;
    }
    hipLaunchKernelGGL(k_ct_tri, dim3(C->g_tri), dim3(128), 0, c->stream, in, C->d_ctl, C->d_ccnt,
                       (const TriRec*)C->d_cand, C->cshard_cap, C->d_item, C->d_par, C->d_head, C->d_blist, C->d_bvel, C->d_lim,
                       C->myu, C->d_evs, C->cap / kEvShards, C->d_ev_nodes, C->d_ev_f);
}

// A2 (multi-GPU): the pair boxes of every rank combined, then this rank's live i-nodes inside
// their range boxes binned into its block
static int xr_a2(hakai_ctx* c, double d_time) {
    Contact* C = c->contact;
    Xrank* X = C->xr;
    hipStream_t s = c->stream;
    const int par = X->par_a, nw = box_words(C->npairs);
    const unsigned gw = (unsigned)((nw + kB - 1) / kB);
    XBox xb{};
    int nxb = 0, flip = 0;
    if (comm_is_rccl(c)) {  // min words as they are, max words complemented: one MIN all-reduce, in place
        hipLaunchKernelGGL(k_xr_boxflip, dim3(gw), dim3(kB), 0, s, X->d_box[par], C->npairs);
        if (int rc = comm_allreduce_min_u64(c, X->d_box[par], X->d_box[par], (size_t)nw)) return rc;
        xb.p[0] = X->d_box[par];
        nxb = 1;
        flip = 1;
    } else {
        for (int q = 0; q < X->nranks; ++q) {
            hakai_ctx* pc = comm_peer_ctx(c, q);
            Xrank* P = pc && pc->contact ? pc->contact->xr : nullptr;
            if (!P || P->seq != X->seq || P->t_a != X->t_a)
                return fail(HAKAI_ERR_STATE, "multi-GPU contact: rank %d has not started step %d", q, X->t_a);
            if (q != X->rank) HIPCHK(hipStreamWaitEvent(s, P->ev_box[par], 0));
            xb.p[q] = P->d_box[par];
        }
        nxb = X->nranks;
    }
    if (C->npairs > kLdsPairs) {  // combined in global memory first
        if (flip) hipLaunchKernelGGL(k_xr_boxflip, dim3(gw), dim3(kB), 0, s, X->d_box[par], C->npairs);
        hipLaunchKernelGGL(k_xr_boxcomb, dim3(gw), dim3(kB), 0, s, xb, nxb, C->npairs, X->d_boxg);
        nxb = 0;
        flip = 0;
    }
    {  // (bin block header zeroed by this step's k_ct_reset)
        StepIn in = step_in(c, X->t_a, d_time);
        hipLaunchKernelGGL(k_xr_bin, dim3((unsigned)std::max(1, C->nseg * C->g_seg)), dim3(kB), 0, s, in,
                           (const Seg*)C->d_seg, C->nseg, C->d_reg, C->d_ni_live, C->d_ni_pair, C->d_ni_node, C->d_par,
                           xb, nxb, flip, C->npairs, X->d_boxg, X->d_send[1][par], X->capq[1][X->rank], C->g_seg);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(X->ev_sent[1][par], s));
    return 0;
}

// A3 (multi-GPU): one hash grid of every rank's binned i-nodes; this rank's own triangles searched
// against it; its events packed for phase B
static int xr_a3(hakai_ctx* c, double d_time) {
    Contact* C = c->contact;
    Xrank* X = C->xr;
    hipStream_t s = c->stream;
    const int par = X->par_a;
    XBlk xb;
    if (int rc = xr_gather(c, 1, par, false, xb)) return rc;
    const unsigned gb = (unsigned)std::min<long long>(std::max<long long>((X->cap[1] + kB - 1) / kB, 1), 128);
    int* hc = X->d_hcnt + (size_t)X->sl_a * Xrank::kNx * X->nranks;
    StepIn in = step_in(c, X->t_a, d_time);
    if (C->n_tri > 0 && C->fuse_binfilter) {  // insert and prefilter side by side
        hipLaunchKernelGGL(k_xr_insfilter, dim3(gb * (unsigned)X->nranks + filter_grid(C)), dim3(kB), 0, s, xb,
                           X->nranks, C->d_par, C->d_ctl, C->d_head, C->d_blist, C->d_bvel, c->d_poison,
                           X->t_a, X->d_xctl, hc, (int)gb, in, C->d_reg + 2 * C->tri_reg + 1, C->d_tri_live,
                           C->d_tri_pair, C->d_tri_nodes, C->d_tri_ele, X->d_boxg, C->d_ccnt, (TriRec*)C->d_cand,
                           C->cshard_cap, C->small ? nullptr : C->d_item);
        tri_search(c, in);
    } else {
        hipLaunchKernelGGL(k_xr_insert, dim3(gb, (unsigned)X->nranks), dim3(kB), 0, s, xb, X->nranks,
                           C->d_par, C->d_ctl, C->d_head, C->d_blist, C->d_bvel, c->d_poison, X->t_a, X->d_xctl, hc);
        if (C->n_tri > 0) {
            tri_prefilter(c, in, X->d_boxg);
            tri_search(c, in);
        }
    }
    hipLaunchKernelGGL(k_ev_pack, dim3((unsigned)C->g_ev), dim3(kB), 0, s, C->d_ctl, C->d_evs, C->cap / kEvShards,
                       C->d_ev_nodes, C->d_ev_f, X->d_send[2][par], X->capq[2][X->rank]);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(X->ev_sent[2][par], s));
    ++X->phase_a;
    C->use_velo0 = false;
    return 0;
}

int contact_phase(hakai_ctx* c, int part, double t, double d_time) {
    Contact* C = c->contact;
    if (!C) return 0;
    if (part == 1) return step_start(c, t, d_time);
    if (!C->xr) return 0;
    return part == 2 ? xr_a2(c, d_time) : xr_a3(c, d_time);
}

int contact_step(hakai_ctx* c, double t, double d_time) {
    if (c->contact && c->contact->xr)
        return fail(HAKAI_ERR_STATE, "contact force probe on a multi-GPU rank: step the group instead");
    return contact_phase(c, 1, t, d_time);
}

bool contact_multi(const hakai_ctx* c) { return c->contact && c->contact->xr; }

// Phase B (multi-GPU): every rank's events -- RCCL all-gather, or the in-process peers' blocks read
// in place -- and the same count / scatter / double-double sums as one GPU, in the global node
// space; the sums of this rank's nodes go to its external force. Also records the step's gathered
// counts for the capacities of later steps.
int contact_step_b(hakai_ctx* c) {
    Contact* C = c->contact;
    Xrank* X = C ? C->xr : nullptr;
    if (!X) return 0;
    hipStream_t s = c->stream;
    const int par = X->par_a, nr = X->nranks;
    XBlk xb;
    if (int rc = xr_gather(c, 2, par, false, xb)) return rc;
    const int tsel = C->tsel;
    const unsigned ge = (unsigned)C->g_ev;
    hipLaunchKernelGGL(k_ct_count_g, dim3(ge), dim3(kB), 0, s, C->d_ctl, xb, nr, X->d_g2l, C->d_cnt,
                       C->d_touched[tsel], C->d_tpos, tsel, c->d_poison, X->t_a, X->d_xctl,
                       X->d_hcnt + (size_t)X->sl_a * Xrank::kNx * nr, C->d_touched[1 - tsel], c->d_fext);
    hipLaunchKernelGGL(k_ct_alloc, dim3(C->g_node), dim3(kB), 0, s, C->d_ctl, tsel, C->d_touched[tsel], C->d_cnt, C->d_toff,
                       C->d_tcnt);
    hipLaunchKernelGGL(k_ct_scatter_g, dim3(ge), dim3(kB), 0, s, xb, nr, X->d_g2l, C->d_ctl, C->d_toff,
                       C->d_tpos, C->d_cnt, C->d_terms);
    hipLaunchKernelGGL(k_ct_sum, dim3(C->g_node), dim3(kB), 0, s, C->d_ctl, tsel, C->d_touched[tsel], C->d_toff, C->d_tcnt,
                       C->d_terms, c->d_fext, X->d_g2l);
    // the step's counts (k_xr_dunpack, k_xr_bcount, k_ct_count_g wrote them into the host-mapped
    // ring slot), read by xr_grow two steps later
    HIPCHK(hipEventRecord(X->ev_cnt[X->sl_a], s));
    ++X->cnt_seq;
    HIPCHK(hipGetLastError());
    return 0;
}

// Graph mode (hakai_step): a step may be captured when its contact work is the same launch sequence
// every step -- one GPU, no full rebuild, no initial velocity, consecutive step numbers.
// contact_step's host state then changes only by the tsel flip and last_t, which
// contact_graph_advance replays for a cached graph's two steps.
bool contact_graph_ok(const hakai_ctx* c, double t) {
    const Contact* C = c->contact;
    if (!C) return true;
    return !C->xr && !C->force_rebuild && !C->always_rebuild && !C->use_velo0 && (long long)t == C->last_t + 1;
}

// hakai_step found a poisoned step: the device state is the last good step's. Rebuild the live
// lists at the next step; velo of the first step is the initial one only if no step survived.
// Multi-GPU: if an exchange capacity overflowed (the same on every rank: they read the same
// headers), grow it past every count of the failed step and pack every deletion step again, so the
// step can run again from there (contact_exchange_retry).
void contact_after_overflow(hakai_ctx* c, long long steps_since_reset) {
    Contact* C = c->contact;
    if (!C) return;
    C->force_rebuild = true;
    C->use_velo0 = steps_since_reset == 0;
    C->last_t = -1;
    if (Xrank* X = C->xr) {
        int xc[4 + 2 * Xrank::kNx * kMaxXRanks] = {0};
        const int nr = X->nranks;
        const size_t n = 4 + 2 * (size_t)Xrank::kNx * nr;
        if (hipMemcpyAsync(xc, X->d_xctl, n * sizeof(int), hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
            hipStreamSynchronize(c->stream) != hipSuccess)
            return;
        X->retry = false;
        if (xc[0] & 7) {  // past the largest count of the call (its steps after the poisoned one included)
            for (int x = 0; x < Xrank::kNx; ++x) {
                if (!(xc[0] & (1 << x))) continue;
                for (int q = 0; q < nr; ++q) {  // every block past its rank's largest count of the call
                    const long long mx = xc[4 + (Xrank::kNx + x) * nr + q];
                    X->capq[x][q] = std::max(X->capq[x][q], xr_cap_target(X, x, mx));
                    int* hq = X->hist[x].data() + (size_t)q * Xrank::kHist;  // (kept by the window)
                    for (int j = 0; j < Xrank::kHist; ++j) hq[j] = std::max<int>(hq[j], (int)std::min<long long>(mx, 1 << 30));
                }
                xr_cap_sums(X, x);
            }
            X->retry = true;
        }
        (void)hipMemsetAsync(X->d_xctl, 0, n * sizeof(int), c->stream);
        if (xr_buffers(c) == 0) (void)xr_dpack(c, true);
    }
}

bool contact_exchange_retry(hakai_ctx* c) {
    Contact* C = c->contact;
    if (!C || !C->xr || !C->xr->retry) return false;
    C->xr->retry = false;
    return true;
}

void contact_graph_advance(hakai_ctx* c, double t_last) {
    Contact* C = c->contact;
    if (!C) return;
    C->last_t = (long long)t_last;  // two steps: tsel flipped twice
}

// candidate buffer of about `total` records in kCandShards shards. A shard holds at least what
// its prefilter blocks can append in one pass over the triangles (kB per block), so a deck whose
// triangles fit one pass of the grid cannot overflow a shard -- as the unsharded n_tri-sized
// buffer could not.
static void size_cand(Contact* C, long long total) {
    const long long blocks = std::max<long long>(1, std::min<long long>((C->n_tri + kB - 1) / kB, kFilterBlocks));
    const long long one_pass = (blocks + kCandShards - 1) / kCandShards * kB;
    C->cshard_cap = std::max<long long>((total + kCandShards - 1) / kCandShards, one_pass);
    C->cand_cap = C->cshard_cap * kCandShards;
}

int contact_tuning(hakai_ctx* c, const char* key, long long value) {
    Contact* C = c->contact;
    if (!C) return fail(HAKAI_ERR_STATE, "%s before set_contact", key);
    if (!std::strcmp(key, "contact_fuse_binfilter")) {
        if (value != 0 && value != 1) return fail(HAKAI_ERR_ARG, "contact_fuse_binfilter must be 0 or 1");
        C->fuse_binfilter = (int)value;
        graph_invalidate(c);
        return 0;
    }
    if (!std::strcmp(key, "contact_fuse_small")) {  // small decks: fused single-workgroup phases
        if (value != 0 && value != 1) return fail(HAKAI_ERR_ARG, "contact_fuse_small must be 0 or 1");
        C->fuse_small = (int)value;
        graph_invalidate(c);
        return 0;
    }
    if (!std::strcmp(key, "contact_candidate_cap")) {
        if (value < 1 || value > (1LL << 31) - 1) return fail(HAKAI_ERR_ARG, "contact_candidate_cap out of range");
        HIPCHK(hipStreamSynchronize(c->stream));
        if (C->d_cand) (void)hipFree(C->d_cand);
        C->d_cand = nullptr;
        dfree(C->d_item);
        size_cand(C, value);
        HIPCHK(hipMalloc(&C->d_cand, (size_t)C->cand_cap * sizeof(TriRec)));
        HIPCHK(dalloc(&C->d_item, (size_t)kItemsPerCand * C->cand_cap));
        HIPCHK(hipMemsetAsync(C->d_ctl + kNcandMax, 0, 3 * sizeof(unsigned int), c->stream));  // + shard max, over
        HIPCHK(hipMemsetAsync(C->d_ctl + kItemShardMax, 0, sizeof(unsigned int), c->stream));
        return 0;
    }
    if (!std::strcmp(key, "contact_exchange_deletions") || !std::strcmp(key, "contact_exchange_bins") ||
        !std::strcmp(key, "contact_exchange_events")) {
        // multi-GPU: records per rank block of an exchange (call on every rank, between steps);
        // capacities also grow on their own, and a step that overflows one runs again (hakai_step)
        Xrank* X = C->xr;
        if (!X) return fail(HAKAI_ERR_STATE, "%s without hakai_set_contact_global", key);
        const int x = key[17] == 'd' ? 0 : (key[17] == 'b' ? 1 : 2);
        if (value < 1 || value > (1LL << 28)) return fail(HAKAI_ERR_ARG, "%s out of range", key);
        HIPCHK(hipDeviceSynchronize());
        for (auto& v : X->capq[x]) v = std::min<long long>(value, X->cap_max[x]);
        X->cap_floor[x] = value;  // (the capacities then follow the counts from there)
        xr_cap_sums(X, x);
        if (int rc = xr_buffers(c)) return rc;
        // the next step's deletion block again, in the new layout (a full block: every rank
        // rebuilds its live lists)
        if (x == 0 && c->state_ok) {
            C->force_rebuild = true;
            return xr_dpack(c, true);
        }
        return 0;
    }
    if (!std::strcmp(key, "contact_full_rebuild")) {
        if (value != 0 && value != 1) return fail(HAKAI_ERR_ARG, "contact_full_rebuild must be 0 or 1");
        C->always_rebuild = value != 0;
        return 0;
    }
    if (!std::strcmp(key, "contact_event_cap")) {
        if (value < 1 || value > (1LL << 30)) return fail(HAKAI_ERR_ARG, "contact_event_cap out of range");
        HIPCHK(hipStreamSynchronize(c->stream));
        dfree(C->d_ev_nodes);
        dfree(C->d_ev_f);
        dfree(C->d_terms);
        dfree(C->d_touched[0]);
        dfree(C->d_touched[1]);
        dfree(C->d_toff);
        dfree(C->d_tcnt);
        C->cap = (value + kEvShards - 1) / kEvShards * kEvShards;
        C->tcap = std::min<long long>(C->nN, 4 * C->cap);
        if (Xrank* X = C->xr) {  // the event block can hold at most the event buffer
            X->cap_max[2] = C->cap;
            for (auto& v : X->capq[2]) v = std::min(v, C->cap);
            xr_cap_sums(X, 2);
        }
        HIPCHK(dalloc(&C->d_ev_nodes, 4 * (size_t)C->cap));
        HIPCHK(dalloc(&C->d_ev_f, 3 * (size_t)C->cap));
        HIPCHK(dalloc(&C->d_terms, 12 * (size_t)C->cap));
        HIPCHK(dalloc(&C->d_touched[0], (size_t)C->tcap));
        HIPCHK(dalloc(&C->d_touched[1], (size_t)C->tcap));
        HIPCHK(dalloc(&C->d_toff, (size_t)C->tcap));
        HIPCHK(dalloc(&C->d_tcnt, (size_t)C->tcap));
        // the previous step's touched list is gone: clear external_force and its count
        HIPCHK(hipMemsetAsync(c->d_fext, 0, 3 * (size_t)c->nN * sizeof(double), c->stream));
        HIPCHK(hipMemsetAsync(C->d_ctl + kTouched, 0, 2 * sizeof(unsigned int), c->stream));
        HIPCHK(hipMemsetAsync(C->d_ctl + kEvMax, 0, sizeof(unsigned int), c->stream));
        HIPCHK(hipMemsetAsync(C->d_ctl + kEvShardMax, 0, sizeof(unsigned int), c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        return 0;
    }
    return fail(HAKAI_ERR_ARG, "unknown tuning key '%s'", key);
}

int contact_check(hakai_ctx* c) {
    Contact* C = c->contact;
    if (!C) return 0;
    unsigned int mx = 0, mc[3] = {0, 0, 0};
    HIPCHK(hipMemcpyAsync(&mx, C->d_ctl + kEvMax, sizeof(unsigned int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(mc, C->d_ctl + kNcandMax, 3 * sizeof(unsigned int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if ((long long)mc[kCandShardMax - kNcandMax] > C->cshard_cap)
        return fail(HAKAI_ERR_STATE, "contact: %u candidate triangles in one step (%u in one of %d shards) exceed the "
                    "buffer (%lld); raise hakai_set_tuning(\"contact_candidate_cap\")", mc[0],
                    mc[kCandShardMax - kNcandMax], kCandShards, C->cand_cap);
    unsigned int mi = 0;  // search items (one per candidate and reachable cell, <= 27 per candidate)
    HIPCHK(hipMemcpy(&mi, C->d_ctl + kItemShardMax, sizeof(unsigned int), hipMemcpyDeviceToHost));
    if ((long long)mi > kItemsPerCand * C->cshard_cap)
        return fail(HAKAI_ERR_STATE, "contact: %u search items in one of %d shards exceed the item buffer (%lld per "
                    "shard, %d per candidate slot); raise hakai_set_tuning(\"contact_candidate_cap\"), which also "
                    "grows the item buffer", mi, kCandShards, (long long)kItemsPerCand * C->cshard_cap, kItemsPerCand);
    if (Xrank* X = C->xr) {
        int xc = 0;
        HIPCHK(hipMemcpy(&xc, X->d_xctl, sizeof(int), hipMemcpyDeviceToHost));
        if (xc & 7)
            return fail(HAKAI_ERR_STATE, "contact exchange: a rank's %s exceeded its block (capacities now %lld / %lld / "
                        "%lld records; grown for the next step)", (xc & 1) ? "deletions" : (xc & 2) ? "binned contact "
                        "nodes" : "events", X->cap[0], X->cap[1], X->cap[2]);
    }
    unsigned int ms = 0;
    HIPCHK(hipMemcpy(&ms, C->d_ctl + kEvShardMax, sizeof(unsigned int), hipMemcpyDeviceToHost));
    if ((long long)ms > C->cap / kEvShards)
        return fail(HAKAI_ERR_STATE, "contact: %u events in one step (%u in one of %d shards) exceed the buffer "
                    "(%lld); raise hakai_set_tuning(\"contact_event_cap\")", mx, ms, kEvShards, C->cap);
    int pz = 0;
    HIPCHK(hipMemcpy(&pz, c->d_poison, sizeof(int), hipMemcpyDeviceToHost));
    if (pz)  // multi-GPU search: another rank's buffers overflowed
        return fail(HAKAI_ERR_STATE, "contact: a contact buffer of another rank overflowed; raise "
                    "hakai_set_tuning(\"contact_event_cap\" / \"contact_candidate_cap\") on every rank");
    return 0;
}

}  // namespace hkc

namespace {

// the mesh contact is set up on: the context's own, or the global one (multi-GPU)
struct HostMesh {
    long long nN, nE;
    const std::vector<double>* coord;  // 3nN
    const std::vector<int>* conn;      // 8nE, 0-based
    const std::vector<int>* mat;       // nE, 0-based
};
// multi-GPU: the entries this rank keeps (owner-computed search, hkc::Xrank) -- the node entries of
// the nodes it owns (node_owner = rank of the node's lowest incident element) with local node ids,
// and the triangles of its elements [E0, E1) with local node and element ids; adders stay global.
struct OwnFilter {
    int rank = 0, nranks = 1;
    const std::vector<int>* node_owner = nullptr;  // [nN global]
    const std::vector<int>* g2l = nullptr;         // [nN global] local node or -1
    long long E0 = 0, E1 = 0;
    std::vector<long long> ni_per_rank;            // out: i-node entries each rank owns
};

// builds c->contact on mesh H (the surfaces, pairs and entry lists of hakai_set_contact_cp);
// contact_flag is 1 or 2, c->contact was destroyed by the caller
int contact_setup(hakai_ctx* c, const HostMesh& H, int32_t contact_flag, const int64_t* element_instance, int32_t n_cp,
                  const int32_t* cp_instance, const int64_t* cp_elem_off, const int64_t* cp_elems, OwnFilter* own) {
    const int nE = (int)H.nE;
    // instances: contiguous element blocks 1, 2, ... (readInpFile numbers them this way)
    std::vector<Inst> inst;
    for (int e = 0; e < nE; ++e) {
        const long long id = element_instance ? element_instance[e] : 1;
        if (id < 1) return fail(HAKAI_ERR_ARG, "element_instance[%d] = %lld", e + 1, id);
        if ((size_t)id > inst.size()) {
            if ((size_t)id != inst.size() + 1)
                return fail(HAKAI_ERR_ARG, "element_instance must number contiguous element blocks 1, 2, ...");
            inst.emplace_back();
            inst.back().e0 = e;
            inst.back().young = c->h_young[(*H.mat)[e]];
        } else if ((size_t)id != inst.size()) {
            return fail(HAKAI_ERR_ARG, "element_instance must number contiguous element blocks 1, 2, ...");
        }
        inst.back().nE++;
    }
    const int ni = (int)inst.size();
    if (ni == 0) return 0;
    for (auto& I : inst) build_instance(I, *H.coord, *H.conn);
    // pairs (:273-311) and CT entries (:332-396). With *Contact Pair surfaces the exterior faces of
    // each side are restricted to the surface's elements (get_surface_triangle's "pick up only
    // contact element", :2087-2112 -- applied only when the list is not the whole instance).
    struct CtDef {
        int a, b;                                  // a: points (i side), b: triangles (j side)
        const std::vector<char>* fa = nullptr;     // element filters (instance-local), null = all
        const std::vector<char>* fb = nullptr;
    };
    std::vector<std::vector<char>> filters;
    filters.reserve(2 * (size_t)n_cp);
    std::vector<std::pair<int, int>> cp;
    std::vector<std::pair<const std::vector<char>*, const std::vector<char>*>> cpf;
    if (n_cp > 0) {
        for (int k = 0; k < n_cp; ++k) {
            const std::vector<char>* f[2] = {nullptr, nullptr};
            int id[2];
            for (int s = 0; s < 2; ++s) {
                id[s] = cp_instance[2 * k + s] - 1;
                if (id[s] < 0 || id[s] >= ni) return fail(HAKAI_ERR_ARG, "contact pair %d: instance %d", k + 1, id[s] + 1);
                const long long b0 = cp_elem_off[2 * k + s], b1 = cp_elem_off[2 * k + s + 1];
                std::vector<char> bm((size_t)inst[id[s]].nE, 0);
                for (long long q = b0; q < b1; ++q) {
                    const long long el = cp_elems[q];
                    if (el < 1 || el > inst[id[s]].nE)
                        return fail(HAKAI_ERR_ARG, "contact pair %d: element %lld not in instance %d", k + 1, el, id[s] + 1);
                    bm[el - 1] = 1;
                }
                if (b1 - b0 != inst[id[s]].nE) {  // the reference compares the list length only (:2087)
                    filters.push_back(std::move(bm));
                    f[s] = &filters.back();
                }
            }
            cp.push_back({id[0], id[1]});
            cpf.push_back({f[0], f[1]});
        }
    } else if (ni > 1) {
        for (int i = 0; i < ni; ++i)
            for (int j = (contact_flag == 2 ? i : i + 1); j < ni; ++j) {
                cp.push_back({i, j});
                cpf.push_back({nullptr, nullptr});
            }
    } else {
        cp.push_back({0, 0});
        cpf.push_back({nullptr, nullptr});
    }
    std::vector<CtDef> ct;
    for (size_t k = 0; k < cp.size(); ++k) {
        ct.push_back({cp[k].first, cp[k].second, cpf[k].first, cpf[k].second});
        if (cp[k].first != cp[k].second) ct.push_back({cp[k].second, cp[k].first, cpf[k].second, cpf[k].first});
    }
    auto* C = new hkc::Contact();
    C->nN = H.nN;
    C->nE = H.nE;
    C->npairs = (int)ct.size();
    // element sizes (:404-421)
    {
#pragma clang fp contract(off)
        double mn = INFINITY, mx = -INFINITY;
        for (int e = 0; e < nE; ++e) {
            const int* el = &(*H.conn)[8 * (size_t)e];
            const double* p1 = &(*H.coord)[3 * (size_t)el[0]];
            const int oth[3] = {1, 3, 4};
            for (int q = 0; q < 3; ++q) {
                const double* p = &(*H.coord)[3 * (size_t)el[oth[q]]];
                const double a = p1[0] - p[0], b = p1[1] - p[1], d = p1[2] - p[2];
                const double L = std::sqrt(a * a + b * b + d * d);
                mn = std::min(mn, L);
                mx = std::max(mx, L);
            }
        }
        C->min_size = mn;
        C->max_size = mx;
        C->d_lim = mn * 0.3;  // :2253
    }
    std::vector<int> ni_pair, ni_node, ni_orig, ni_aptr{0}, ni_add;
    std::vector<int> nj_pair, nj_node, nj_orig, nj_aptr{0}, nj_add;
    std::vector<int> tri_pair, tri_nodes, tri_ele, tri_adder, seg;
    struct SegKey {
        int inst;
        const void* filt;
        int adds;
    };
    std::vector<SegKey> seg_key;
    // node list of a pair side: initial exterior nodes + nodes exposed by each element's deletion
    auto keep = [](const Inst& I, const std::vector<char>* filt, int f) {
        return !filt || (*filt)[I.faces[f].ele - I.e0];
    };
    if (own) own->ni_per_rank.assign((size_t)own->nranks, 0);
    auto node_list = [&](int pr, const Inst& I, const std::vector<char>* filt, bool with_adds, std::vector<int>& vp,
                         std::vector<int>& vn, std::vector<int>& vo, std::vector<int>& va, std::vector<int>& vadd,
                         bool side_i) {
        // per node: initial (exterior) or the ascending list of elements whose deletion exposes it;
        // bucketed by node id in linear time (adders arrive in ascending element order)
        const int nN = (int)H.nN;
        std::vector<char> orig((size_t)nN, 0), seen((size_t)nN, 0);
        for (int f : I.exterior)
            if (keep(I, filt, f))
                for (int q = 0; q < 4; ++q) orig[I.faces[f].n[q]] = seen[I.faces[f].n[q]] = 1;
        std::vector<int> cnt((size_t)nN + 1, 0), adders;
        if (with_adds) {
            for (int j = 0; j < I.nE; ++j)
                for (int f : I.added[j])
                    for (int q = 0; q < 4; ++q) {
                        const int n = I.faces[f].n[q];
                        seen[n] = 1;
                        if (!orig[n]) cnt[n + 1]++;
                    }
            for (int n = 0; n < nN; ++n) cnt[n + 1] += cnt[n];
            adders.resize((size_t)cnt[nN]);
            std::vector<int> fill(cnt.begin(), cnt.end() - 1);
            for (int j = 0; j < I.nE; ++j)
                for (int f : I.added[j])
                    for (int q = 0; q < 4; ++q) {
                        const int n = I.faces[f].n[q];
                        if (!orig[n]) adders[fill[n]++] = I.e0 + j;
                    }
        }
        long long count = 0;
        for (int n = 0; n < nN; ++n) {
            if (!seen[n]) continue;
            if (own) {
                const int q = (*own->node_owner)[n];
                if (side_i) own->ni_per_rank[q]++;
                if (q != own->rank) {
                    count += orig[n];
                    continue;
                }
            }
            vp.push_back(pr);
            vn.push_back(own ? (*own->g2l)[n] : n);
            vo.push_back(orig[n]);
            if (!orig[n] && with_adds) {
                int last = -1;
                for (int a = cnt[n]; a < cnt[n + 1]; ++a)
                    if (adders[a] != last) vadd.push_back(last = adders[a]);  // duplicates are adjacent
            }
            va.push_back((int)vadd.size());
            count += orig[n];
        }
        return count;
    };
    int hoff = 0;
    for (int pr = 0; pr < C->npairs; ++pr) {
        const int a = ct[pr].a, b = ct[pr].b;  // a: points (i), b: triangles (j)
        const bool self = a == b;
        PairParam pp;
        pp.young = inst[b].young;  // :367
        pp.self = self;
        pp.kc = self ? C->kc_s : C->kc_o;
        pp.Cr = self ? C->Cr_s : C->Cr_o;
        pp.ddiv = self ? C->max_size * 0.6 : C->max_size * 1.1;  // :2322-2325
        const size_t ni0 = ni_node.size(), nj0 = nj_node.size();
        // surface update (:766-804): c_nodes_i grows for every pair whose point instance lost an
        // element; triangles and c_nodes_j grow only when the triangle instance differs
        const long long c_i = node_list(pr, inst[a], ct[pr].fa, true, ni_pair, ni_node, ni_orig, ni_aptr, ni_add, true);
        const long long c_j =
            node_list(pr, inst[b], ct[pr].fb, !self, nj_pair, nj_node, nj_orig, nj_aptr, nj_add, false);
        long long c_t = 0;
        // a triangle (:2140-2145) of element ele, exposed from the start (adder -1) or by the deletion
        // of adder; multi-GPU: kept by the rank of ele, with local ids
        auto add_tri = [&](const int* n, int ele, int adder) {
            const int tv[6] = {n[0], n[1], n[2], n[2], n[3], n[0]};
            const bool mine = !own || (ele >= own->E0 && ele < own->E1);
            for (int h = 0; h < 2; ++h) {
                if (!mine) continue;
                tri_pair.push_back(pr);
                for (int q = 0; q < 3; ++q) tri_nodes.push_back(own ? (*own->g2l)[tv[3 * h + q]] : tv[3 * h + q]);
                tri_ele.push_back(own ? (int)(ele - own->E0) : ele);
                tri_adder.push_back(adder);
            }
        };
        for (int f : inst[b].exterior) {
            if (!keep(inst[b], ct[pr].fb, f)) continue;
            add_tri(inst[b].faces[f].n, inst[b].faces[f].ele, -1);
            c_t += 2;
        }
        if (!self)
            for (int j = 0; j < inst[b].nE; ++j)
                for (int f : inst[b].added[j]) add_tri(inst[b].faces[f].n, inst[b].faces[f].ele, inst[b].e0 + j);
        // a segment's live node set is a function of (instance, face filter, adders or not): equal
        // keys, equal sets at every step, so one segment's boxes serve both
        if (ni_node.size() > ni0) {
            seg.insert(seg.end(), {(int)ni0, (int)ni_node.size(), pr, 0, -1, 0, -1, -1});
            seg_key.push_back({a, (const void*)ct[pr].fa, 1});
        }
        if (nj_node.size() > nj0) {
            seg.insert(seg.end(), {(int)nj0, (int)nj_node.size(), pr, 1, -1, 0, -1, -1});
            seg_key.push_back({b, (const void*)ct[pr].fb, self ? 0 : 1});
        }
        // sized for the initial surface; nodes exposed later share buckets (slower, same result)
        int hs = 64;
        while (hs < 2 * c_i) hs <<= 1;
        pp.hash_off = hoff;
        pp.hash_size = hs;
        hoff += hs;
        C->h_par.push_back(pp);
        C->pair_inst.push_back(a + 1);
        C->pair_inst.push_back(b + 1);
        C->pair_counts.push_back(c_i);
        C->pair_counts.push_back(c_t);
        C->pair_counts.push_back(c_j);
    }
    C->htot = hoff;
    C->n_ni = (int)ni_node.size();
    C->n_nj = (int)nj_node.size();
    C->n_tri = (int)tri_ele.size();
    C->nseg = (int)seg.size() / 8;
    for (int q = 0; q < C->nseg; ++q)  // bounding-box duplicates (Seg::dup / alias)
        for (int r = 0; r < q; ++r) {
            const SegKey &x = seg_key[q], &y = seg_key[r];
            if (seg[8 * r + 5] || x.inst != y.inst || x.filt != y.filt || x.adds != y.adds) continue;
            int* al = &seg[8 * r + 6];
            const int k = al[0] < 0 ? 0 : (al[1] < 0 ? 1 : -1);
            if (k < 0) break;  // r already serves two: q computes its own
            al[k] = 12 * seg[8 * q + 2] + 6 * seg[8 * q + 3];
            seg[8 * q + 5] = 1;
            break;
        }
    // fused small-deck phases: one 1024-thread workgroup scans the deletion steps, the bucket table
    // and the i-node entries a few times at most
    C->small = C->nE <= (1 << 16) && C->n_ni <= (1 << 16) && C->htot <= (1 << 15);
    {  // event buffer: 8 events per initial contact point (overflow is detected and reported)
        long long ci0 = 0;
        for (int p = 0; p < C->npairs; ++p) ci0 += C->pair_counts[3 * p];
        C->cap = std::max<long long>(1 << 16, 8LL * ci0);
        C->cap = (C->cap + kEvShards - 1) / kEvShards * kEvShards;
    }
    C->tcap = std::min<long long>(H.nN, 4 * C->cap);
    {  // launch grids (see Contact::g_*): large models keep the full grids
        auto clampi = [](long long v, long long lo, long long hi) { return (int)std::max(lo, std::min(hi, v)); };
        long long ci0 = 0, ct0 = 0, maxseg = 1;
        for (int p = 0; p < C->npairs; ++p) {
            ci0 += C->pair_counts[3 * p];
            ct0 += C->pair_counts[3 * p + 1];
        }
        for (int q = 0; q < C->nseg; ++q) maxseg = std::max<long long>(maxseg, seg[8 * q + 1] - seg[8 * q]);
        C->g_seg = clampi((maxseg + kB - 1) / kB, 1, kSegBlocks);
        C->g_box = clampi((maxseg + 4 * kB - 1) / (4 * kB), 1, 128);  // ~4 entries per thread: one unrolled pass
        C->g_ev = clampi((4 * ci0 + kB - 1) / kB, 16, 1024);
        // >= 64 waves (every event shard); one pass over 16 search items (reachable cells) per live
        // triangle up to the 4096-block cap -- small self-contact decks keep half their triangles
        C->g_tri = clampi(((C->small ? 32 : 16) * ct0 + 127) / 128, 32, 4096);  // (small: 32 lanes per candidate)
        C->g_node = clampi((2 * ci0 + kB - 1) / kB, 4, 256);
        C->g_del = clampi((C->nE / 4 + kB - 1) / kB, 1, 1024);
        C->g_reset = clampi((std::max<long long>(std::max<long long>(kEvShards, 12LL * C->npairs), 2 * ci0) + kB - 1) / kB,
                            1, 64);
    }
    // live-list regions: i-node segments, j-node segments, then the triangle list; tiles of
    // kTile entries inside one region each (full rebuild)
    std::vector<Tile> tiles;
    std::vector<int> reg_first, reg;  // reg: [nreg][2] (base, count = 0)
    std::vector<int> pair_reg(2 * (size_t)C->npairs, -1);
    auto add_region = [&](int list, int a0, int a1) {
        const int r = (int)reg_first.size();
        reg_first.push_back((int)tiles.size());
        C->reg_list_h.push_back(list);
        reg.push_back(a0);
        reg.push_back(0);
        for (int k = a0; k < a1; k += kTile) tiles.push_back({list, k, std::min(a1, k + kTile), r});
        return r;
    };
    for (int list = 0; list < 2; ++list)
        for (int q = 0; q < C->nseg; ++q)
            if (seg[8 * q + 3] == list) {
                const int r = add_region(list, seg[8 * q], seg[8 * q + 1]);
                seg[8 * q + 4] = r;
                pair_reg[2 * (size_t)seg[8 * q + 2] + list] = r;
            }
    C->tri_reg = add_region(2, 0, C->n_tri);
    C->nreg = (int)reg_first.size();
    reg_first.push_back((int)tiles.size());
    C->ntile = (int)tiles.size();
    // element -> entries its deletion exposes (CSR over global element ids)
    auto invert = [&](const std::vector<int>& aptr, const std::vector<int>& add, int n, std::vector<int>& ptr,
                      std::vector<int>& idx) {
        ptr.assign((size_t)nE + 1, 0);
        for (int k = 0; k < n; ++k)
            for (int a = aptr[k]; a < aptr[k + 1]; ++a) ptr[add[a] + 1]++;
        for (int e = 0; e < nE; ++e) ptr[e + 1] += ptr[e];
        idx.resize((size_t)ptr[nE]);
        std::vector<int> fill(ptr.begin(), ptr.end() - 1);
        for (int k = 0; k < n; ++k)
            for (int a = aptr[k]; a < aptr[k + 1]; ++a) idx[fill[add[a]]++] = k;
    };
    std::vector<int> el_ni_ptr, el_ni, el_nj_ptr, el_nj, el_tri_ptr, el_tri;
    invert(ni_aptr, ni_add, C->n_ni, el_ni_ptr, el_ni);
    invert(nj_aptr, nj_add, C->n_nj, el_nj_ptr, el_nj);
    {
        std::vector<int> taptr((size_t)C->n_tri + 1, 0), tadd;
        for (int j = 0; j < C->n_tri; ++j) {
            if (tri_adder[j] >= 0) tadd.push_back(tri_adder[j]);
            taptr[j + 1] = (int)tadd.size();
        }
        invert(taptr, tadd, C->n_tri, el_tri_ptr, el_tri);
    }
    hipStream_t s = c->stream;
    int rc = 0;
#define UP(dst, v)                                          \
    do {                                                    \
        hipError_t _e = upload(&C->dst, v, s);              \
        if (_e != hipSuccess) rc = hip_fail(_e, #dst);      \
    } while (0)
    UP(d_par, C->h_par);
    UP(d_seg, seg);
    UP(d_ni_pair, ni_pair); UP(d_ni_node, ni_node); UP(d_ni_orig, ni_orig); UP(d_ni_aptr, ni_aptr); UP(d_ni_add, ni_add);
    UP(d_nj_pair, nj_pair); UP(d_nj_node, nj_node); UP(d_nj_orig, nj_orig); UP(d_nj_aptr, nj_aptr); UP(d_nj_add, nj_add);
    UP(d_tri_pair, tri_pair); UP(d_tri_nodes, tri_nodes); UP(d_tri_ele, tri_ele); UP(d_tri_adder, tri_adder);
    UP(d_reg_first, reg_first); UP(d_reg, reg); UP(d_pair_reg, pair_reg);
    UP(d_el_ni_ptr, el_ni_ptr); UP(d_el_ni, el_ni); UP(d_el_nj_ptr, el_nj_ptr); UP(d_el_nj, el_nj);
    UP(d_el_tri_ptr, el_tri_ptr); UP(d_el_tri, el_tri);
    {
        Tile* dt = nullptr;
        hipError_t e = upload(&dt, tiles, s);
        C->d_tiles = dt;
        if (e != hipSuccess) rc = hip_fail(e, "d_tiles");
    }
#undef UP
    c->contact = C;
    if (rc) {
        hkc::contact_destroy(c);
        return rc;
    }
    HIPCHK(dalloc(&C->d_head, (size_t)C->htot));
    HIPCHK(hipMemsetAsync(C->d_head, 0, (size_t)C->htot * sizeof(unsigned long long), s));  // stamp 0: empty
    C->blist_cap = std::max(C->n_ni, 1);  // (multi-GPU: sized for every rank's records, xr_buffers)
    HIPCHK(dalloc(&C->d_blist, (size_t)C->blist_cap));
    HIPCHK(dalloc(&C->d_bvel, (size_t)C->blist_cap));
    HIPCHK(dalloc(&C->d_tile_cnt, (size_t)C->ntile));
    HIPCHK(dalloc(&C->d_tile_off, (size_t)C->ntile + 1));
    HIPCHK(dalloc(&C->d_dlist, (size_t)nE));
    HIPCHK(dalloc(&C->d_ni_live, (size_t)C->n_ni));
    HIPCHK(dalloc(&C->d_nj_live, (size_t)C->n_nj));
    HIPCHK(dalloc(&C->d_tri_live, (size_t)C->n_tri));
    HIPCHK(dalloc(&C->d_bbox, (size_t)box_words(C->npairs)));
    HIPCHK(dalloc(&C->d_ctl, (size_t)kCtl));
    HIPCHK(dalloc(&C->d_evs, (size_t)kEvShards * kShardStride));
    HIPCHK(hipMemsetAsync(C->d_evs, 0, (size_t)kEvShards * kShardStride * sizeof(unsigned int), s));
    HIPCHK(dalloc(&C->d_ev_nodes, 4 * (size_t)C->cap));
    HIPCHK(dalloc(&C->d_ev_f, 3 * (size_t)C->cap));
    HIPCHK(dalloc(&C->d_cnt, (size_t)H.nN + 1));
    HIPCHK(dalloc(&C->d_tpos, (size_t)H.nN + 1));
    HIPCHK(dalloc(&C->d_touched[0], (size_t)C->tcap));
    HIPCHK(dalloc(&C->d_touched[1], (size_t)C->tcap));
    HIPCHK(dalloc(&C->d_toff, (size_t)C->tcap));
    HIPCHK(dalloc(&C->d_tcnt, (size_t)C->tcap));
    {
        long long t0 = 0;  // initial live triangles
        for (int p = 0; p < C->npairs; ++p) t0 += C->pair_counts[3 * p + 1];
        size_cand(C, std::min<long long>(std::max<long long>(C->n_tri, 1), std::max<long long>(1 << 16, 4 * t0)));
    }
    HIPCHK(dalloc(&C->d_ccnt, (size_t)kCandShards * kShardStride));
    HIPCHK(hipMalloc(&C->d_cand, (size_t)C->cand_cap * sizeof(TriRec)));
    HIPCHK(dalloc(&C->d_item, (size_t)kItemsPerCand * C->cand_cap));
    if (C->htot >= (1 << 27)) return fail(HAKAI_ERR_ARG, "contact: %d hash buckets (search items hold 27 bits)", C->htot);
    HIPCHK(dalloc(&C->d_terms, 12 * (size_t)C->cap));
    HIPCHK(dalloc(&C->d_velo0, 3 * (size_t)c->nN));
    HIPCHK(dalloc(&c->d_fext, 3 * (size_t)c->nN));
    HIPCHK(hipMemsetAsync(C->d_cnt, 0, ((size_t)H.nN + 1) * sizeof(int), s));
    HIPCHK(hipMemsetAsync(C->d_ctl, 0, kCtl * sizeof(unsigned int), s));
    HIPCHK(hipMemsetAsync(c->d_fext, 0, 3 * (size_t)c->nN * sizeof(double), s));
    C->force_rebuild = true;
    // velocity before the first step: the state's (IC / uploaded) velocity (local nodes)
    if (!c->h_velo0.empty())
        HIPCHK(hipMemcpyAsync(C->d_velo0, c->h_velo0.data(), 3 * (size_t)c->nN * sizeof(double), hipMemcpyHostToDevice, s));
    else
        HIPCHK(hipMemsetAsync(C->d_velo0, 0, 3 * (size_t)c->nN * sizeof(double), s));
    C->use_velo0 = c->steps_done == 0 || !c->h_velo0.empty();
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

// Multi-GPU (hkc::Xrank) for a contact set up on the global mesh with this rank's entries: the
// node maps, the global mass and deletion arrays, the exchange blocks; packs the first deletion
// block if a state exists.
int xr_build(hakai_ctx* c, const OwnFilter& own, long long nNode, long long nElement, const double* diag_M,
             const std::vector<int>& g2l, const int64_t* local_node_global, const int64_t* rank_elem_off) {
    hkc::Contact* C = c->contact;
    auto* X = new hkc::Xrank();
    C->xr = X;
    const int nr = own.nranks;
    X->rank = own.rank;
    X->nranks = nr;
    X->E0 = own.E0;
    X->nEloc = own.E1 - own.E0;
    X->nN_g = nNode;
    X->nE_g = nElement;
    std::vector<long long> eoff((size_t)nr + 1);
    for (int q = 0; q <= nr; ++q) eoff[q] = rank_elem_off[q];
    for (int q = 0; q < nr; ++q) X->maxEloc = std::max<int>(X->maxEloc, (int)(eoff[q + 1] - eoff[q]));
    long long ci0 = 0, nimax = 1;
    for (int p = 0; p < C->npairs; ++p) ci0 += C->pair_counts[3 * p];
    for (long long v : own.ni_per_rank) nimax = std::max(nimax, v);
    // capacities (records per rank block): deletions up to a rank's elements, binned i-nodes up to
    // the entries a rank owns, events up to the event buffer; they start small and grow
    X->cap_max[0] = X->maxEloc;
    X->cap_max[1] = nimax;
    X->cap_max[2] = C->cap;
    const long long cap0[hkc::Xrank::kNx] = {std::min<long long>(X->cap_max[0], 1024),
                                        std::min<long long>(X->cap_max[1], std::max<long long>(4096, ci0 / (8 * nr))),
                                        std::min<long long>(X->cap_max[2], 4096)};
    for (int x = 0; x < hkc::Xrank::kNx; ++x) {
        X->capq[x].assign((size_t)nr, cap0[x]);
        X->hist[x].assign((size_t)nr * hkc::Xrank::kHist, 0);
        xr_cap_sums(X, x);
    }
    std::vector<int> l2g((size_t)c->nN);
    for (long long l = 0; l < c->nN; ++l) l2g[l] = (int)(local_node_global[l] - 1);
    std::vector<double> gmass((size_t)nNode);
    for (long long n = 0; n < nNode; ++n) gmass[n] = diag_M[3 * n];
    hipStream_t s = c->stream;
    HIPCHK(upload(&X->d_l2g, l2g, s));
    HIPCHK(upload(&X->d_g2l, g2l, s));
    HIPCHK(upload(&X->g_mass, gmass, s));
    HIPCHK(upload(&X->d_eoff, eoff, s));
    HIPCHK(dalloc(&X->g_del, (size_t)nElement + 2));
    HIPCHK(hipMemsetAsync(X->g_del, 0, ((size_t)nElement + 2) * sizeof(int), s));
    HIPCHK(dalloc(&X->d_last_del, (size_t)std::max<long long>(X->nEloc, 1)));
    HIPCHK(hipMemsetAsync(X->d_last_del, 0, (size_t)std::max<long long>(X->nEloc, 1) * sizeof(int), s));
    HIPCHK(dalloc(&X->d_xctl, 4 + 2 * (size_t)hkc::Xrank::kNx * nr));
    HIPCHK(hipMemsetAsync(X->d_xctl, 0, (4 + 2 * (size_t)hkc::Xrank::kNx * nr) * sizeof(int), s));
    for (int p = 0; p < 2; ++p) {
        HIPCHK(dalloc(&X->d_box[p], (size_t)box_words(C->npairs)));
        HIPCHK(hipEventCreateWithFlags(&X->ev_box[p], hipEventDisableTiming));
        for (int x = 0; x < hkc::Xrank::kNx; ++x) HIPCHK(hipEventCreateWithFlags(&X->ev_sent[x][p], hipEventDisableTiming));
    }
    HIPCHK(dalloc(&X->d_boxg, (size_t)box_words(C->npairs)));
    HIPCHK(hipHostMalloc((void**)&X->h_cnt, 4 * (size_t)hkc::Xrank::kNx * nr * sizeof(int),
                         hipHostMallocMapped | hipHostMallocCoherent));
    std::fill(X->h_cnt, X->h_cnt + 4 * (size_t)hkc::Xrank::kNx * nr, 0);
    HIPCHK(hipHostGetDevicePointer((void**)&X->d_hcnt, X->h_cnt, 0));
    for (auto& e : X->ev_cnt) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIPCHK(hipStreamSynchronize(s));
    if (int rc = hkc::xr_buffers(c)) return rc;
    if (c->state_ok)
        if (int rc = hkc::contact_state_reset(c, c->h_velo0.empty() ? nullptr : c->h_velo0.data())) return rc;
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

}  // namespace

extern "C" {

int hakai_set_contact(hakai_ctx* c, int32_t contact_flag, const int64_t* element_instance) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    return hakai_set_contact_cp(c, contact_flag, element_instance, 0, nullptr, nullptr, nullptr);
}

int hakai_set_contact_cp(hakai_ctx* c, int32_t contact_flag, const int64_t* element_instance, int32_t n_cp,
                         const int32_t* cp_instance, const int64_t* cp_elem_off, const int64_t* cp_elems) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    if (n_cp < 0 || (n_cp > 0 && (!cp_instance || !cp_elem_off || !cp_elems)))
        return fail(HAKAI_ERR_ARG, "set_contact_cp: bad contact-pair arrays");
    if (!c->model_ok) return fail(HAKAI_ERR_STATE, "set_contact before upload_model");
    HIPCHK(hipSetDevice(c->device));
    hkc::contact_destroy(c);
    if (contact_flag < 1) return 0;
    if (contact_flag > 2) return fail(HAKAI_ERR_ARG, "contact_flag %d (0, 1 or 2)", contact_flag);
    if (c->comm)
        return fail(HAKAI_ERR_STATE, "contact on a rank of a multi-GPU group: use hakai_set_contact_global");
    const HostMesh H{c->nN, c->nE, &c->h_coord, &c->h_conn, &c->h_mat};
    return contact_setup(c, H, contact_flag, element_instance, n_cp, cp_instance, cp_elem_off, cp_elems, nullptr);
}

int hakai_set_contact_global(hakai_ctx* c, int32_t contact_flag, int64_t nNode, const double* coordmat,
                             int64_t nElement, const int64_t* elementmat, const int64_t* element_material,
                             const int64_t* element_instance, const double* diag_M, const int64_t* local_node_global,
                             const int64_t* rank_elem_off, int32_t n_cp, const int32_t* cp_instance,
                             const int64_t* cp_elem_off, const int64_t* cp_elems) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    if (n_cp < 0 || (n_cp > 0 && (!cp_instance || !cp_elem_off || !cp_elems)))
        return fail(HAKAI_ERR_ARG, "set_contact_global: bad contact-pair arrays");
    if (!c->model_ok) return fail(HAKAI_ERR_STATE, "set_contact_global before upload_model");
    if (!c->comm) return fail(HAKAI_ERR_STATE, "set_contact_global before comm_init / comm_init_local");
    HIPCHK(hipSetDevice(c->device));
    hkc::contact_destroy(c);
    if (contact_flag < 1) return 0;
    if (contact_flag > 2) return fail(HAKAI_ERR_ARG, "contact_flag %d (0, 1 or 2)", contact_flag);
    if (nNode <= 0 || nElement <= 0 || !coordmat || !elementmat || !element_material || !diag_M ||
        !local_node_global || !rank_elem_off)
        return fail(HAKAI_ERR_ARG, "set_contact_global: bad arguments");
    if (nNode >= (int64_t)INT32_MAX || 8 * nElement >= (int64_t)INT32_MAX)
        return fail(HAKAI_ERR_ARG, "set_contact_global: mesh too large for int32 indexing");
    const int nr = hkc::comm_size(c), rank = hkc::comm_rank(c);
    if (rank_elem_off[0] != 0 || rank_elem_off[nr] != nElement)
        return fail(HAKAI_ERR_ARG, "set_contact_global: rank_elem_off must run from 0 to nElement");
    for (int q = 0; q < nr; ++q)
        if (rank_elem_off[q + 1] < rank_elem_off[q]) return fail(HAKAI_ERR_ARG, "set_contact_global: rank_elem_off decreases");
    if (rank_elem_off[rank] != c->elem_offset || rank_elem_off[rank + 1] - rank_elem_off[rank] != c->nE)
        return fail(HAKAI_ERR_ARG, "set_contact_global: rank %d holds elements %lld..+%lld, rank_elem_off says %lld..%lld",
                    rank, c->elem_offset, c->nE, (long long)rank_elem_off[rank], (long long)rank_elem_off[rank + 1]);
    std::vector<double> gx(coordmat, coordmat + 3 * nNode);
    std::vector<int> gconn(8 * (size_t)nElement), gmat((size_t)nElement);
    for (int64_t e = 0; e < nElement; ++e) {
        for (int i = 0; i < 8; ++i) {
            const int64_t n = elementmat[8 * e + i];
            if (n < 1 || n > nNode) return fail(HAKAI_ERR_ARG, "set_contact_global: elementmat[%d,%lld] = %lld", i + 1, (long long)e + 1, (long long)n);
            gconn[8 * e + i] = (int)(n - 1);
        }
        const int64_t m = element_material[e];
        if (m < 1 || m > c->nmat) return fail(HAKAI_ERR_ARG, "set_contact_global: element_material[%lld] = %lld", (long long)e + 1, (long long)m);
        gmat[e] = (int)(m - 1);
    }
    // local -> global nodes, checked against this rank's uploaded connectivity
    std::vector<int> g2l((size_t)nNode, -1);
    for (long long l = 0; l < c->nN; ++l) {
        const int64_t g = local_node_global[l];
        if (g < 1 || g > nNode || g2l[g - 1] >= 0)
            return fail(HAKAI_ERR_ARG, "set_contact_global: local_node_global[%lld] = %lld", l + 1, (long long)g);
        g2l[g - 1] = (int)l;
    }
    for (long long e = 0; e < c->nE; ++e)
        for (int i = 0; i < 8; ++i)
            if (gconn[8 * (c->elem_offset + e) + i] != local_node_global[c->h_conn[8 * e + i]] - 1)
                return fail(HAKAI_ERR_ARG, "set_contact_global: local element %lld differs from global element %lld", e + 1,
                            c->elem_offset + e + 1);
    if (nr > hkc::kMaxXRanks) return fail(HAKAI_ERR_ARG, "set_contact_global: more than %d ranks", hkc::kMaxXRanks);
    // owner of a node: the rank of its lowest incident element (ranks hold ascending element ranges)
    std::vector<int> minel((size_t)nNode, INT32_MAX), owner((size_t)nNode, -1);
    for (int64_t e = 0; e < nElement; ++e)
        for (int i = 0; i < 8; ++i) {
            int& m = minel[gconn[8 * e + i]];
            m = std::min(m, (int)e);
        }
    for (int64_t n = 0; n < nNode; ++n)
        if (minel[n] != INT32_MAX) {
            const int q = (int)(std::upper_bound(rank_elem_off, rank_elem_off + nr + 1, (int64_t)minel[n]) - rank_elem_off) - 1;
            owner[n] = q;
            if (q == rank && g2l[n] < 0)
                return fail(HAKAI_ERR_ARG, "set_contact_global: owned node %lld is not in the local model", (long long)n + 1);
        }
    OwnFilter own;
    own.rank = rank;
    own.nranks = nr;
    own.node_owner = &owner;
    own.g2l = &g2l;
    own.E0 = rank_elem_off[rank];
    own.E1 = rank_elem_off[rank + 1];
    const HostMesh H{nNode, nElement, &gx, &gconn, &gmat};
    int rc = contact_setup(c, H, contact_flag, element_instance, n_cp, cp_instance, cp_elem_off, cp_elems, &own);
    if (rc || !c->contact) return rc;
    rc = xr_build(c, own, nNode, nElement, diag_M, g2l, local_node_global, rank_elem_off);
    if (rc) hkc::contact_destroy(c);
    return rc;
}

int hakai_set_contact_params(hakai_ctx* c, double myu, double kc_o, double kc_s, double Cr_o, double Cr_s) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    hkc::Contact* C = c->contact;
    if (!C) return fail(HAKAI_ERR_STATE, "set_contact_params before set_contact");
    C->myu = myu;
    C->kc_o = kc_o;
    C->kc_s = kc_s;
    C->Cr_o = Cr_o;
    C->Cr_s = Cr_s;
    for (auto& p : C->h_par) {
        p.kc = p.self ? kc_s : kc_o;
        p.Cr = p.self ? Cr_s : Cr_o;
    }
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemcpyAsync(C->d_par, C->h_par.data(), C->h_par.size() * sizeof(PairParam), hipMemcpyHostToDevice,
                          c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int hakai_contact_info(hakai_ctx* c, int32_t* n_pairs, int64_t* info, int32_t cap, double* sizes) {
    if (!c || !n_pairs) return fail(HAKAI_ERR_ARG, "null");
    hkc::Contact* C = c->contact;
    *n_pairs = C ? C->npairs : 0;
    if (!C) return 0;
    for (int p = 0; p < C->npairs && p < cap; ++p) {
        info[5 * p + 0] = C->pair_inst[2 * p];
        info[5 * p + 1] = C->pair_inst[2 * p + 1];
        info[5 * p + 2] = C->pair_counts[3 * p];
        info[5 * p + 3] = C->pair_counts[3 * p + 1];
        info[5 * p + 4] = C->pair_counts[3 * p + 2];
    }
    if (sizes) {
        sizes[0] = C->min_size;
        sizes[1] = C->max_size;
    }
    return 0;
}

int hakai_contact_stats(hakai_ctx* c, int64_t* stats, int32_t cap) {
    if (!c || (!stats && cap > 0)) return fail(HAKAI_ERR_ARG, "null");
    hkc::Contact* C = c->contact;
    if (!C) return fail(HAKAI_ERR_STATE, "contact_stats before set_contact");
    HIPCHK(hipSetDevice(c->device));
    std::vector<unsigned int> ctl(kCtl);
    std::vector<int> reg(2 * (size_t)C->nreg);
    HIPCHK(hipMemcpyAsync(ctl.data(), C->d_ctl, kCtl * sizeof(unsigned int), hipMemcpyDeviceToHost, c->stream));
    if (C->nreg)
        HIPCHK(hipMemcpyAsync(reg.data(), C->d_reg, reg.size() * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    long long live[3] = {0, 0, 0};
    const int64_t v[7] = {ctl[kEv], ctl[kEvMax], ctl[kNcand], ctl[kTouched + C->tsel], 0, 0, 0};
    for (int r = 0; r < C->nreg; ++r) live[C->reg_list_h[r]] += reg[2 * r + 1];
    for (int k = 0; k < cap && k < 7; ++k) stats[k] = k < 4 ? v[k] : live[k == 4 ? 2 : k - 5];
    long long rec_bytes = 0;
    if (cap > 7) {  // multi-GPU: contact-zone i-nodes all ranks binned in the last step; the bytes this
                    // rank's exchanges receive per step (the other ranks' blocks at their capacities)
                    // and the bytes of the records in them (headers + the last step's gathered counts)
        long long binned = 0, bytes = 0;
        if (hkc::Xrank* X = C->xr) {
            const int nr = X->nranks;
            std::vector<int> cnt((size_t)hkc::Xrank::kNx * nr);
            HIPCHK(hipMemcpy(cnt.data(), X->d_xctl + 4, cnt.size() * sizeof(int), hipMemcpyDeviceToHost));
            for (int q = 0; q < nr; ++q) binned += cnt[(size_t)nr + q];
            for (int x = 0; x < hkc::Xrank::kNx; ++x)
                for (int q = 0; q < nr; ++q) {
                    if (q == X->rank) continue;
                    bytes += (long long)hkc::xr_blkq(X, x, q);
                    rec_bytes += (long long)kXHdr + (long long)hkc::xr_rec_bytes(x) * cnt[(size_t)x * nr + q];
                }
        }
        stats[7] = binned;
        if (cap > 8) stats[8] = bytes;
    }
    if (cap > 9) stats[9] = C->htot;  // hash-grid buckets over all pairs
    if (cap > 10) {  // live triangles the prefilter tested in full (those with a non-empty range box)
        std::vector<unsigned int> cc((size_t)kCandShards * kShardStride);
        HIPCHK(hipMemcpy(cc.data(), C->d_ccnt, cc.size() * sizeof(unsigned int), hipMemcpyDeviceToHost));
        long long nt = 0;
        for (int q = 0; q < kCandShards; ++q) nt += cc[(size_t)q * kShardStride + kTestWord];
        stats[10] = nt;
    }
    if (cap > 11) stats[11] = rec_bytes;
    return 0;
}

int hakai_contact_force(hakai_ctx* c, double t, double d_time, double* external_force) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c || !external_force) return fail(HAKAI_ERR_ARG, "null");
    if (!c->contact) return fail(HAKAI_ERR_STATE, "contact_force before set_contact");
    if (!c->state_ok) return fail(HAKAI_ERR_STATE, "contact_force before reset/upload_state");
    HIPCHK(hipSetDevice(c->device));
    const bool keep = c->contact->use_velo0;
    c->contact->force_rebuild = true;  // live lists for this t; and again for the next real step
    int rc = hkc::contact_step(c, t, d_time);
    c->contact->use_velo0 = keep;  // a probe, not a step
    c->contact->force_rebuild = true;
    if (rc) return rc;
    HIPCHK(hipMemcpyAsync(external_force, c->d_fext, 3 * (size_t)c->nN * sizeof(double), hipMemcpyDeviceToHost,
                          c->stream));
    HIPCHK(hipMemsetAsync(c->d_poison, 0, 2 * sizeof(int), c->stream));  // a probe changes no state
    HIPCHK(hipStreamSynchronize(c->stream));
    return hkc::contact_check(c);
}

}  // extern "C"
