// hakai_capi.cpp -- C ABI of libhakai_hip.so (declared in include/hakai_hip.h).
//
// Owns the persistent device context: model, Gauss-point state in SoA, ping-pong displacement
// buffers, the node->element incidence CSR used for the deterministic force gather, BC tables,
// deletion log and per-kernel HIP-event timers. One HIP stream per context.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/hakai_hip.h"
#include "hakai_internal.hpp"
#include "hakai_kernels.hpp"

using hk::DevMat;

namespace {
thread_local std::string g_err;
}

namespace hkc {

int fail(int code, const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_fail(hipError_t e, const char* what) {
    return fail(HAKAI_ERR_DEVICE, "%s: %s", what, hipGetErrorString(e));
}

}  // namespace hkc

using hkc::fail;
using hkc::hip_fail;

#define HIPCHK(x)                                           \
    do {                                                    \
        hipError_t _e = (x);                                \
        if (_e != hipSuccess) return hip_fail(_e, #x);      \
    } while (0)

template <class T>
static hipError_t dalloc(T** p, size_t n) {
    *p = nullptr;
    if (n == 0) n = 1;
    return hipMalloc((void**)p, n * sizeof(T));
}

template <class T>
static void dfree(T*& p) {
    if (p) (void)hipFree((void*)p);
    p = nullptr;
}

namespace hkc {

static void own_free(hakai_ctx* c) {
    dfree(c->d_own_off);
    dfree(c->d_own_seq);
    dfree(c->d_own_bstart);
    dfree(c->d_own_list);
    dfree(c->d_own_q);
    dfree(c->d_own_rp);
    dfree(c->d_own_rows);
    dfree(c->d_own_ridx);
    dfree(c->d_own_dump);
    c->own_built_g = -1;
    c->own_for_g0 = -1;
    c->own_valid = false;
}

static void free_model(hakai_ctx* c) {
    contact_destroy(c);
    dfree(c->d_coord);
    dfree(c->d_u[0]);
    dfree(c->d_u[1]);
    dfree(c->d_mass);
    dfree(c->d_conn);
    dfree(c->d_flag);
    dfree(c->d_mat);
    dfree(c->d_mats);
    dfree(c->d_stress);
    dfree(c->d_strain);
    dfree(c->d_eqps);
    dfree(c->d_yield);
    dfree(c->d_triax);
    dfree(c->d_fe);
    dfree(c->d_inc_ptr);
    dfree(c->d_inc);
    dfree(c->d_inc_row);
    dfree(c->d_inc8);
    dfree(c->d_del_step);
    dfree(c->d_qbuf);
    dfree(c->d_fext);
    own_free(c);
    c->model_ok = false;
    c->state_ok = false;
}

static void free_bc(hakai_ctx* c) {
    dfree(c->d_bc_of_node);
    dfree(c->d_bc_dof);
    dfree(c->d_bc_grp);
    dfree(c->d_bc_val);
    dfree(c->d_amp_n);
    dfree(c->d_amp_off);
    dfree(c->d_amp_t);
    dfree(c->d_amp_v);
    c->nbc = 0;
}

// Material constants exactly as hakai() derives them (v2/HAKAI_j.jl:143-160) and readInpFile
// builds Hd (v2/readInpFile_j.jl:763-768).
int build_devmat(const hakai_material_t& in, DevMat& o) {
    std::memset(&o, 0, sizeof o);
    const double young = in.young, poisson = in.poisson;
    const double d1 = (1.0 - poisson), d2 = poisson, d3 = (1.0 - 2.0 * poisson) / 2.0;
    const double cc = young / (1.0 + poisson) / (1.0 - 2.0 * poisson);
    o.Dn = cc * d1;
    o.Do = cc * d2;
    o.Ds = cc * d3;
    o.G = young / 2. / (1.0 + poisson);
    o.density = in.density;
    if (in.n_plastic < 0 || in.n_plastic > hk::kMaxPlastic)
        return fail(HAKAI_ERR_ARG, "material: %d plastic rows (max %d)", in.n_plastic, hk::kMaxPlastic);
    if (in.n_ductile < 0 || in.n_ductile > hk::kMaxDuctile)
        return fail(HAKAI_ERR_ARG, "material: %d ductile rows (max %d)", in.n_ductile, hk::kMaxDuctile);
    if (in.n_plastic == 1)
        return fail(HAKAI_ERR_MODEL,
                    "material: a single *Plastic row gives an empty Hd; the reference raises BoundsError "
                    "(v2/HAKAI_j.jl:1267)");
    o.npp = in.n_plastic;
    o.nd = in.n_ductile;
    o.yield0 = in.n_plastic > 0 ? in.plastic[0] : 0.0;
    for (int r = 0; r < in.n_plastic; ++r) o.pl_eps[r] = in.plastic[2 * r + 1];
    for (int r = 0; r + 1 < in.n_plastic; ++r)
        o.Hd[r] = (in.plastic[2 * (r + 1)] - in.plastic[2 * r]) / (in.plastic[2 * (r + 1) + 1] - in.plastic[2 * r + 1]);
    for (int r = 0; r < in.n_ductile; ++r) {
        o.du_eps[r] = in.ductile[3 * r + 0];
        o.du_tri[r] = in.ductile[3 * r + 1];
    }
    // ductile_fr returns a table value or a linear interpolation between two neighbouring ones,
    // i.e. at least the smallest fracture strain less a few rounding errors of its terms: an element
    // average below min - (|max| + |min|) * 2^-40 cannot reach it, and the kernels skip the table
    // search (the same deletion decisions, tests/test_gpu_exact.py, test_gpu_fullsize.py)
    double lo = 0.0, hi = 0.0;
    for (int r = 0; r < in.n_ductile; ++r) {
        lo = r == 0 ? o.du_eps[r] : std::min(lo, o.du_eps[r]);
        hi = r == 0 ? o.du_eps[r] : std::max(hi, o.du_eps[r]);
    }
    o.du_floor = in.n_ductile > 0 ? lo - (std::fabs(hi) + std::fabs(lo)) * 0x1p-40 : 0.0;
    if (!(o.du_floor == o.du_floor)) o.du_floor = -HUGE_VAL;  // (a NaN table: never skip)
    // an element average of eight values below du_skip (rounded sums: at most 8 ulps above their
    // bound) stays below du_floor: a wave whose Gauss points all lie below it needs no averages
    o.du_skip = o.du_floor > 0.0 ? o.du_floor - o.du_floor * 0x1p-40 : -HUGE_VAL;
    return 0;
}

// cal_Pusai_hexa (v2/HAKAI_j.jl:1895-1943): dN_i/dxi at the 8 Gauss points, out[24k + 8r + i],
// with the reference's expression order (this file is compiled without contraction).
void pusai_table(double out[192]) {
    static const double delta[8][3] = {{-1.0, -1.0, -1.0}, {1.0, -1.0, -1.0}, {1.0, 1.0, -1.0}, {-1.0, 1.0, -1.0},
                                       {-1.0, -1.0, 1.0},  {1.0, -1.0, 1.0},  {1.0, 1.0, 1.0},  {-1.0, 1.0, 1.0}};
    const double g = 1.0 / std::sqrt(3.0);
    for (int k = 0; k < 8; ++k) {  // gc order :1913-1920: k bits = (xi, eta, zeta) signs
        const double gzai = (k & 4) ? g : -g, eta = (k & 2) ? g : -g, tueta = (k & 1) ? g : -g;
        for (int i = 0; i < 8; ++i) {
            out[24 * k + i] = 1.0 / 8.0 * delta[i][0] * (1.0 + eta * delta[i][1]) * (1.0 + tueta * delta[i][2]);
            out[24 * k + 8 + i] = 1.0 / 8.0 * delta[i][1] * (1.0 + gzai * delta[i][0]) * (1.0 + tueta * delta[i][2]);
            out[24 * k + 16 + i] = 1.0 / 8.0 * delta[i][2] * (1.0 + gzai * delta[i][0]) * (1.0 + eta * delta[i][1]);
        }
    }
}

hipStream_t ctx_stream(hakai_ctx* c) { return c->stream; }
int ctx_device(hakai_ctx* c) { return c->device; }

}  // namespace hkc

// ---------------------------------------------------------------------------------------------
// profiling
// ---------------------------------------------------------------------------------------------
static void prof_harvest(hakai_ctx* c) {
    if (c->ev_pending.empty()) return;
    (void)hipEventSynchronize(c->ev_pending.back().b);
    for (auto& p : c->ev_pending) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
            c->k_ms[p.kernel] += ms;
            c->k_n[p.kernel] += 1;
        }
        c->ev_pool.push_back(p.a);
        c->ev_pool.push_back(p.b);
    }
    c->ev_pending.clear();
}

static hipEvent_t prof_event(hakai_ctx* c) {
    if (c->ev_pool.empty()) {
        if (c->ev_pending.size() >= 2048) prof_harvest(c);
        if (c->ev_pool.empty()) {
            hipEvent_t e;
            (void)hipEventCreate(&e);
            return e;
        }
    }
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
}

namespace hkc {
void prof_begin(hakai_ctx* c, int kernel, EventPair* p) {
    p->kernel = -1;
    if (!c->prof || !((c->prof_mask >> kernel) & 1u)) return;
    p->kernel = kernel;
    p->a = prof_event(c);
    p->b = prof_event(c);
    (void)hipEventRecord(p->a, c->stream);
}
void prof_end(hakai_ctx* c, EventPair* p) {
    if (!c->prof || p->kernel < 0) return;
    (void)hipEventRecord(p->b, c->stream);
    c->ev_pending.push_back(*p);
}
void graph_invalidate(hakai_ctx* c) {
    c->epoch++;
    c->tdev_next = -1;
}
static void graph_free(hakai_ctx* c) {
    for (int g = 0; g < 2; ++g)
        for (int p = 0; p < 2; ++p)
            if (c->g_exec[g][p]) {
                (void)hipGraphExecDestroy(c->g_exec[g][p]);
                c->g_exec[g][p] = nullptr;
                c->g_epoch[g][p] = -1;
            }
}
}  // namespace hkc


// Kernel arguments of the element update for the context's current buffers.
static hk::ElemArgs elem_args(hakai_ctx* c) {
    hk::ElemArgs ea;
    std::memset(&ea, 0, sizeof ea);
    ea.coord = c->d_coord;
    ea.u = c->d_u[c->cur];
    ea.u_pre = c->d_u[1 - c->cur];
    ea.conn = c->d_conn;
    ea.flag = c->d_flag;
    ea.mat = c->d_mat;
    ea.mats = c->d_mats;
    ea.stress = c->d_stress;
    ea.strain = c->d_strain;
    for (int q = 0; q < 6; ++q) {
        ea.sc[q] = c->d_stress + q * c->ld;
        ea.ec[q] = c->d_strain + q * c->ld;
    }
    ea.eqps = c->d_eqps;
    ea.yield = c->d_yield;
    ea.triax = c->d_triax;
    ea.fe = c->d_fe;
    ea.vol = nullptr;
    ea.nE = c->nE;
    ea.nEp = c->nEp;
    ea.ld = c->ld;
    ea.del_step = c->d_del_step;
    ea.step_i = 0;
    ea.any_plastic = c->any_plastic ? 1 : 0;
    // nEp / 32 = batches of 32 elements (kEPB); small meshes take the one-batch-per-block kernel
    ea.pipe_blocks = (c->nEp / 32 >= (long long)c->pipe_min * c->pipe_blocks) ? c->pipe_blocks : 0;
    ea.gp_nt = c->gp_nt;
    ea.nmat = c->nmat;
    ea.exact = c->elem_exact;
    ea.pusai = c->d_pusai;
    ea.poison = c->d_poison;
    return ea;
}

// Element forces [nEp][8][3] <-> the reference's Qe (24 x nE): the same layout.
static int fe_download_qe(hakai_ctx* c, double* Qe) {
    HIPCHK(hipMemcpyAsync(Qe, c->d_fe, 24 * (size_t)c->nE * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

static int fe_upload_qe(hakai_ctx* c, const double* Qe) {
    HIPCHK(hipMemcpyAsync(c->d_fe, Qe, 24 * (size_t)c->nE * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

// Incidence tables (CSR and padded) as force row bases 24e + 3k; padding -> the zero base 24nEp.
static int fe_upload_incidence(hakai_ctx* c) {
    std::vector<int> inc(c->h_inc0.size());
    for (size_t j = 0; j < inc.size(); ++j) inc[j] = 24 * (c->h_inc0[j] >> 3) + 3 * (c->h_inc0[j] & 7);
    if (!inc.empty())
        HIPCHK(hipMemcpyAsync(c->d_inc, inc.data(), inc.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    if (c->d_inc8) {
        std::vector<int> inc8(8 * (size_t)c->nN, (int)(24 * c->nEp));
        for (long long n = 0; n < c->nN; ++n)
            for (int j = c->h_ptr[n]; j < c->h_ptr[n + 1]; ++j) inc8[8 * n + (j - c->h_ptr[n])] = inc[j];
        HIPCHK(hipMemcpyAsync(c->d_inc8, inc8.data(), inc8.size() * sizeof(int), hipMemcpyHostToDevice, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

// ---------------------------------------------------------------------------------------------
extern "C" {

int hakai_abi_version(void) { return HAKAI_ABI_VERSION; }
const char* hakai_last_error(void) { return g_err.c_str(); }

int hakai_device_count(int* n) {
    if (!n) return fail(HAKAI_ERR_ARG, "null");
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess) cnt = 0;
    *n = cnt;
    return 0;
}

int hakai_create(hakai_ctx** out, int device) {
    if (!out) return fail(HAKAI_ERR_ARG, "null ctx pointer");
    *out = nullptr;
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= 0)
        return fail(HAKAI_ERR_DEVICE, "no HIP device visible: the HAKAI MI355X path has no CPU fallback");
    if (device < 0 || device >= cnt) return fail(HAKAI_ERR_ARG, "device %d out of range (%d visible)", device, cnt);
    HIPCHK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(HAKAI_ERR_DEVICE, "device %d is %s; libhakai_hip is built for gfx950 only", device,
                    prop.gcnArchName);
    hakai_ctx* c = new hakai_ctx();
    c->device = device;
    if (const char* v = std::getenv("HAKAI_PIPE_BLOCKS")) c->pipe_blocks = std::atoi(v);
    // HAKAI_GRAPH=n: steps per captured graph (0 = stream mode). rocprofv3 --kernel-trace crashes
    // the host process on any hipGraph launch with this ROCm (tools/graph_probe.hip alone
    // reproduces it), so the profiling scripts run with HAKAI_GRAPH=0.
    if (const char* v = std::getenv("HAKAI_GRAPH")) {
        const int g = std::atoi(v);
        c->graph = (g >= 0 && g <= 1024 && !(g & 1)) ? g : 0;
    }
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete c;
        return hip_fail(e, "hipStreamCreate");
    }
    if (dalloc(&c->d_negjac, 1) != hipSuccess || dalloc(&c->d_pusai, 192) != hipSuccess ||
        dalloc(&c->d_poison, 2) != hipSuccess || hipMemset(c->d_poison, 0, 2 * sizeof(int)) != hipSuccess) {
        dfree(c->d_negjac);
        dfree(c->d_pusai);
        dfree(c->d_poison);
        delete c;
        return fail(HAKAI_ERR_DEVICE, "hipMalloc for context bookkeeping failed");
    }
    {
        double pus[192];
        hkc::pusai_table(pus);
        // the reference-order element step forms each P2 product once per partner pair and takes
        // the partner's as its exact negation (elem_step_exact): the table must be odd in each sign
        bool odd = true;
        for (int k = 0; k < 8; ++k)
            for (int i = 0; i < 8; ++i) {
                const double* p = pus + 24 * k;
                odd = odd && p[i] == -p[i ^ 1] && p[8 + i] == -p[8 + (i ^ 3)] && p[16 + i] == -p[16 + (i ^ 4)];
            }
        e = odd ? hipMemcpy(c->d_pusai, pus, sizeof pus, hipMemcpyHostToDevice) : hipErrorInvalidValue;
        if (e != hipSuccess) {
            dfree(c->d_negjac);
            dfree(c->d_pusai);
            dfree(c->d_poison);
            delete c;
            return hip_fail(e, "hipMemcpy (Pusai table)");
        }
    }
    if (const char* v = std::getenv("HAKAI_ELEM_EXACT")) c->elem_exact = std::atoi(v) ? 1 : 0;
    if (const char* v = std::getenv("HAKAI_OWN_ASSEMBLY")) c->own_assembly = std::atoi(v) ? 1 : 0;
    *out = c;
    return 0;
}

int hakai_destroy(hakai_ctx* c) {
    if (!c) return 0;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    prof_harvest(c);
    hkc::graph_free(c);
    dfree(c->d_tstep);
    hkc::comm_destroy(c);
    hkc::free_model(c);
    hkc::free_bc(c);
    dfree(c->d_negjac);
    dfree(c->d_pusai);
    dfree(c->d_poison);
    for (auto e : c->ev_pool) (void)hipEventDestroy(e);
    (void)hipStreamDestroy(c->stream);
    delete c;
    return 0;
}

int hakai_upload_model(hakai_ctx* c, int64_t nNode, const double* coordmat, int64_t nElement,
                       const int64_t* elementmat, const int64_t* element_material, int32_t nMat,
                       const hakai_material_t* mats, const double* diag_M) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c) return fail(HAKAI_ERR_ARG, "null ctx");
    if (nNode <= 0 || nElement < 0 || !coordmat || (nElement > 0 && (!elementmat || !element_material)) || nMat <= 0 ||
        !mats || !diag_M)
        return fail(HAKAI_ERR_ARG, "upload_model: bad arguments");
    if (26 * (nElement + 32) + 8 >= (int64_t)INT32_MAX || nNode >= (int64_t)INT32_MAX)
        return fail(HAKAI_ERR_ARG, "upload_model: mesh too large for int32 indexing on one rank");
    // the element kernel addresses its arrays with a 32-bit byte offset per lane (the element
    // forces, 192 B per element, are the largest): at most ~22 M hex per context; larger meshes
    // are split over ranks (hakai_comm_init / hakai_comm_init_local, also on one GPU)
    if (192 * (nElement + 32) >= (int64_t)1 << 32)
        return fail(HAKAI_ERR_ARG, "upload_model: %lld elements exceed one context's 32-bit element-kernel offsets "
                    "(max %lld); split the mesh over ranks", (long long)nElement, (long long)(((int64_t)1 << 32) / 192 - 32));
    // (node gathers: 24 B per node, load_node / load_node_raw form 24u * n)
    if (24 * (nNode + 1) >= (int64_t)1 << 32)
        return fail(HAKAI_ERR_ARG, "upload_model: %lld nodes exceed one context's 32-bit element-kernel offsets "
                    "(max %lld); split the mesh over ranks", (long long)nNode, (long long)(((int64_t)1 << 32) / 24 - 1));
    HIPCHK(hipSetDevice(c->device));
    (void)hipStreamSynchronize(c->stream);
    hkc::free_model(c);
    // BC tables are sized for the previous mesh (the fused-BC per-dof table has 3nN entries): a new
    // model starts without BCs until hakai_set_bc runs again
    hkc::free_bc(c);
    const long long nN = nNode, nE = nElement;
    const long long nEp = ((nE + 31) / 32) * 32;  // whole 32-element batches; padding behaves as deleted
    // host-side conversions
    std::vector<int> conn((size_t)(8 * nEp), 0), mat((size_t)nEp, 0);
    for (long long e = 0; e < nE; ++e) {
        for (int i = 0; i < 8; ++i) {
            const int64_t n = elementmat[8 * e + i];
            if (n < 1 || n > nN) return fail(HAKAI_ERR_ARG, "elementmat[%d,%lld] = %lld out of 1..%lld", i + 1, e + 1, (long long)n, nN);
            conn[8 * e + i] = (int)(n - 1);
        }
        const int64_t m = element_material[e];
        if (m < 1 || m > nMat) return fail(HAKAI_ERR_ARG, "element_material[%lld] = %lld out of 1..%d", e + 1, (long long)m, nMat);
        mat[e] = (int)(m - 1);
    }
    std::vector<double> mass((size_t)nN);
    for (long long n = 0; n < nN; ++n) {
        const double m0 = diag_M[3 * n], m1 = diag_M[3 * n + 1], m2 = diag_M[3 * n + 2];
        if (!(m0 == m1 && m1 == m2))
            return fail(HAKAI_ERR_ARG, "diag_M: node %lld has different masses per dof", n + 1);
        mass[n] = m0;
    }
    c->h_mats.assign((size_t)nMat, DevMat());
    c->nmat = nMat;
    c->has_ductile = false;
    for (int i = 0; i < nMat; ++i) {
        int r = hkc::build_devmat(mats[i], c->h_mats[i]);
        if (r) return r;
    }
    c->any_plastic = false;
    for (long long e = 0; e < nE; ++e) {
        if (c->h_mats[mat[e]].nd > 0) c->has_ductile = true;
        if (c->h_mats[mat[e]].npp > 0) c->any_plastic = true;
    }
    // node -> (8e+i) incidence CSR in ascending element order (counting sort keeps the order)
    std::vector<int> ptr((size_t)nN + 1, 0), inc((size_t)(8 * nE));
    for (long long j = 0; j < 8 * nE; ++j) ptr[conn[j] + 1]++;
    for (long long n = 0; n < nN; ++n) ptr[n + 1] += ptr[n];
    {
        std::vector<int> fill(ptr.begin(), ptr.end() - 1);
        for (long long j = 0; j < 8 * nE; ++j) inc[fill[conn[j]]++] = (int)j;
    }
    int maxinc = 0;
    for (long long n = 0; n < nN; ++n) maxinc = std::max(maxinc, ptr[n + 1] - ptr[n]);
    c->nN = nN;
    c->nE = nE;
    c->nEp = nEp;
    c->ld = 8 * nEp;
    const size_t ld = (size_t)c->ld;
    HIPCHK(dalloc(&c->d_coord, 3 * (size_t)nN));
    HIPCHK(dalloc(&c->d_u[0], 3 * (size_t)nN));
    HIPCHK(dalloc(&c->d_u[1], 3 * (size_t)nN));
    HIPCHK(dalloc(&c->d_mass, (size_t)nN));
    HIPCHK(dalloc(&c->d_conn, 8 * (size_t)nEp));
    HIPCHK(dalloc(&c->d_flag, (size_t)nEp));
    HIPCHK(dalloc(&c->d_mat, (size_t)nEp));
    HIPCHK(dalloc(&c->d_del_step, (size_t)nEp + 2));
    HIPCHK(dalloc(&c->d_mats, (size_t)nMat));
    HIPCHK(dalloc(&c->d_stress, 6 * ld));
    HIPCHK(dalloc(&c->d_strain, 6 * ld));
    HIPCHK(dalloc(&c->d_eqps, ld));
    HIPCHK(dalloc(&c->d_yield, ld));
    HIPCHK(dalloc(&c->d_triax, ld));
    // forces: 24nEp doubles in either layout, then zeros up to 26nEp (padding base 24nEp with
    // component stride up to nEp)
    c->fe_len = 26 * nEp + 8;
    HIPCHK(dalloc(&c->d_fe, (size_t)c->fe_len));
    HIPCHK(dalloc(&c->d_inc_ptr, (size_t)nN + 1));
    HIPCHK(dalloc(&c->d_inc, 8 * (size_t)nE));
    HIPCHK(dalloc(&c->d_inc_row, 8 * (size_t)nE));
    HIPCHK(dalloc(&c->d_qbuf, 3 * (size_t)nN));
    hipStream_t s = c->stream;
    HIPCHK(hipMemcpyAsync(c->d_coord, coordmat, 3 * nN * sizeof(double), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->d_mass, mass.data(), nN * sizeof(double), hipMemcpyHostToDevice, s));
    if (nE) {
        HIPCHK(hipMemcpyAsync(c->d_conn, conn.data(), 8 * nEp * sizeof(int), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->d_mat, mat.data(), nEp * sizeof(int), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->d_inc_row, inc.data(), 8 * nE * sizeof(int), hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipMemcpyAsync(c->d_mats, c->h_mats.data(), nMat * sizeof(DevMat), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->d_inc_ptr, ptr.data(), (nN + 1) * sizeof(int), hipMemcpyHostToDevice, s));
    if (maxinc <= 8) HIPCHK(dalloc(&c->d_inc8, 8 * (size_t)nN));  // padded table for the unrolled gather
    HIPCHK(hipStreamSynchronize(s));  // host vectors go out of scope
    c->max_inc = maxinc;
    c->h_ptr = ptr;
    c->h_inc0 = inc;
    {
        int r = fe_upload_incidence(c);
        if (r) return r;
    }
    c->h_coord.assign(coordmat, coordmat + 3 * nN);
    c->h_conn.assign(conn.begin(), conn.begin() + 8 * nE);
    c->h_mat.assign(mat.begin(), mat.begin() + nE);
    c->h_young.resize((size_t)nMat);
    for (int i = 0; i < nMat; ++i) c->h_young[i] = mats[i].young;
    c->model_ok = true;
    c->state_ok = false;
    return hakai_reset_state(c, 0, nullptr, nullptr, 1.0);
}

int hakai_set_bc(hakai_ctx* c, const hakai_bc_t* bc) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c || !bc) return fail(HAKAI_ERR_ARG, "null");
    if (!c->model_ok) return fail(HAKAI_ERR_STATE, "set_bc before upload_model");
    HIPCHK(hipSetDevice(c->device));
    (void)hipStreamSynchronize(c->stream);
    hkc::free_bc(c);
    const int G = bc->n_groups;
    if (G <= 0) return 0;
    // Resolve in-order overwrites: final writer of each dof (v2/HAKAI_j.jl:585-617).
    std::map<long long, std::pair<int, double>> last;
    for (int g = 0; g < G; ++g) {
        if (bc->amp_n[g] == 1)
            return fail(HAKAI_ERR_MODEL, "BC group %d: one-point amplitude, the reference raises BoundsError (:598)", g + 1);
        for (int64_t en = bc->entry_off[g]; en < bc->entry_off[g + 1]; ++en)
            for (int64_t d = bc->dof_off[en]; d < bc->dof_off[en + 1]; ++d) {
                const int64_t dof = bc->dofs[d];
                if (dof < 1 || dof > 3 * c->nN) return fail(HAKAI_ERR_ARG, "BC dof %lld out of range", (long long)dof);
                last[dof - 1] = std::make_pair(g, bc->entry_value[en]);
            }
    }
    std::vector<int> dof, grp;
    std::vector<double> val;
    for (auto& kv : last) {
        dof.push_back((int)kv.first);
        grp.push_back(kv.second.first);
        val.push_back(kv.second.second);
    }
    std::vector<int> amp_n(G), amp_off(G);
    long long n_amp = 0;
    for (int g = 0; g < G; ++g) {
        amp_n[g] = bc->amp_n[g];
        amp_off[g] = (int)bc->amp_off[g];
        n_amp = std::max<long long>(n_amp, bc->amp_off[g] + bc->amp_n[g]);
    }
    c->nbc = (int)dof.size();
    HIPCHK(dalloc(&c->d_bc_dof, dof.size()));
    HIPCHK(dalloc(&c->d_bc_grp, grp.size()));
    HIPCHK(dalloc(&c->d_bc_val, val.size()));
    HIPCHK(dalloc(&c->d_amp_n, (size_t)G));
    HIPCHK(dalloc(&c->d_amp_off, (size_t)G));
    HIPCHK(dalloc(&c->d_amp_t, (size_t)n_amp));
    HIPCHK(dalloc(&c->d_amp_v, (size_t)n_amp));
    hipStream_t s = c->stream;
    if (!dof.empty()) {
        HIPCHK(hipMemcpyAsync(c->d_bc_dof, dof.data(), dof.size() * sizeof(int), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->d_bc_grp, grp.data(), grp.size() * sizeof(int), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->d_bc_val, val.data(), val.size() * sizeof(double), hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipMemcpyAsync(c->d_amp_n, amp_n.data(), G * sizeof(int), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(c->d_amp_off, amp_off.data(), G * sizeof(int), hipMemcpyHostToDevice, s));
    if (n_amp) {
        HIPCHK(hipMemcpyAsync(c->d_amp_t, bc->amp_time, n_amp * sizeof(double), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(c->d_amp_v, bc->amp_value, n_amp * sizeof(double), hipMemcpyHostToDevice, s));
    }
    // per-node table: the first resolved entry of each node (entries are sorted by dof, a node's
    // up-to-3 entries are consecutive) or -1, so the nodal kernel applies the BCs itself
    // (hakai_step; 4 B per node)
    if (!dof.empty()) {  // (used by k_nodal up to kFuseBcMaxNodes, and by the two-step schedule)
        std::vector<int> of((size_t)c->nN, -1);
        for (size_t i = dof.size(); i-- > 0;) of[(size_t)dof[i] / 3] = (int)i;
        HIPCHK(dalloc(&c->d_bc_of_node, of.size()));
        HIPCHK(hipMemcpyAsync(c->d_bc_of_node, of.data(), of.size() * sizeof(int), hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

int hakai_reset_state(hakai_ctx* c, int64_t n_ic, const int64_t* ic_dofs, const double* ic_values, double d_time) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (c) c->own_valid = false;  // the next nodal update gathers fe (or the uploaded Q)
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    if (!c->model_ok) return fail(HAKAI_ERR_STATE, "reset_state before upload_model");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const size_t fn = 3 * (size_t)c->nN;
    c->cur = 0;
    HIPCHK(hipMemsetAsync(c->d_u[0], 0, fn * sizeof(double), s));
    HIPCHK(hipMemsetAsync(c->d_u[1], 0, fn * sizeof(double), s));
    HIPCHK(hipMemsetAsync(c->d_fe, 0, (size_t)c->fe_len * sizeof(double), s));
    HIPCHK(hipMemsetAsync(c->d_del_step, 0, ((size_t)c->nEp + 2) * sizeof(int), s));
    HIPCHK(hk::launch_reset_gp(c->d_stress, c->d_strain, c->d_eqps, c->d_yield, c->d_triax, c->d_flag, c->d_mat,
                               c->d_mats, c->nE, c->nEp, c->ld, s));
    c->h_velo0.assign(fn, 0.0);
    c->q_from_buf = false;
    c->fe_ok = c->triax_ok = true;
    c->steps_done = 0;
    HIPCHK(hipMemsetAsync(c->d_poison, 0, 2 * sizeof(int), s));
    hkc::comm_reset(c);
    if (n_ic > 0) {
        if (!ic_dofs || !ic_values) return fail(HAKAI_ERR_ARG, "reset_state: null IC arrays");
        std::vector<double> dpre(fn, 0.0);
        for (int64_t j = 0; j < n_ic; ++j) {  // v2/HAKAI_j.jl:233-239
            const int64_t d = ic_dofs[j];
            if (d < 1 || d > (int64_t)fn) return fail(HAKAI_ERR_ARG, "IC dof %lld out of range", (long long)d);
            dpre[d - 1] = -ic_values[j] * d_time;
            c->h_velo0[d - 1] = ic_values[j];
        }
        HIPCHK(hipMemcpyAsync(c->d_u[1 - c->cur], dpre.data(), fn * sizeof(double), hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    c->state_ok = true;
    if (int r = hkc::contact_state_reset(c, c->h_velo0.data())) return r;
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

static int own_materialize(hakai_ctx* c);

int hakai_upload_state(hakai_ctx* c, const hakai_state_t* st) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c || !st) return fail(HAKAI_ERR_ARG, "null");
    if (!c->model_ok) return fail(HAKAI_ERR_STATE, "upload_state before upload_model");
    HIPCHK(hipSetDevice(c->device));
    // The next nodal update gathers fe unless the upload brings Q or Qe. After a call whose last
    // steps a contact overflow skipped, owner-computed assembly left the last element step's forces
    // only as node sums (fe is an earlier step's): they become the uploaded Q, the same bits, and an
    // upload that also deletes elements (whose fe rows it would zero) must bring Q or Qe itself.
    if (c->own_valid && !c->fe_ok && !st->Q && !st->Qe) {
        bool dels = false;
        for (long long e = 0; st->element_flag && e < c->nE && !dels; ++e) dels = st->element_flag[e] == 0;
        if (dels || c->comm)
            return fail(HAKAI_ERR_STATE, "upload_state: the last element step's forces exist only as owner-computed "
                        "node sums (a contact overflow skipped the call's last step); upload Q (from "
                        "hakai_download_state) or Qe with this state");
        if (int r = own_materialize(c)) return r;
    }
    c->own_valid = false;
    hipStream_t s = c->stream;
    const size_t fn = 3 * (size_t)c->nN, nGP = 8 * (size_t)c->nE;
    if (st->disp) HIPCHK(hipMemcpyAsync(c->d_u[c->cur], st->disp, fn * sizeof(double), hipMemcpyHostToDevice, s));
    if (st->disp_pre)
        HIPCHK(hipMemcpyAsync(c->d_u[1 - c->cur], st->disp_pre, fn * sizeof(double), hipMemcpyHostToDevice, s));
    if (st->velo) c->h_velo0.assign(st->velo, st->velo + fn);
    if (st->Q) {
        HIPCHK(hipMemcpyAsync(c->d_qbuf, st->Q, fn * sizeof(double), hipMemcpyHostToDevice, s));
        c->q_from_buf = true;
    }
    if (st->integ_stress || st->integ_strain) {
        double* tmp = nullptr;
        HIPCHK(dalloc(&tmp, 6 * nGP));
        if (st->integ_stress) {
            HIPCHK(hipMemcpyAsync(tmp, st->integ_stress, 6 * nGP * sizeof(double), hipMemcpyHostToDevice, s));
            HIPCHK(hk::launch_aos_to_soa6(tmp, c->d_stress, (long long)nGP, c->ld, s));
        }
        if (st->integ_strain) {
            HIPCHK(hipMemcpyAsync(tmp, st->integ_strain, 6 * nGP * sizeof(double), hipMemcpyHostToDevice, s));
            HIPCHK(hk::launch_aos_to_soa6(tmp, c->d_strain, (long long)nGP, c->ld, s));
        }
        HIPCHK(hipStreamSynchronize(s));
        dfree(tmp);
    }
    if (st->integ_yield_stress)
        HIPCHK(hipMemcpyAsync(c->d_yield, st->integ_yield_stress, nGP * sizeof(double), hipMemcpyHostToDevice, s));
    if (st->integ_eq_plastic_strain)
        HIPCHK(hipMemcpyAsync(c->d_eqps, st->integ_eq_plastic_strain, nGP * sizeof(double), hipMemcpyHostToDevice, s));
    if (st->integ_triax_stress)
        HIPCHK(hipMemcpyAsync(c->d_triax, st->integ_triax_stress, nGP * sizeof(double), hipMemcpyHostToDevice, s));
    if (st->element_flag) {
        std::vector<int> f((size_t)c->nE);
        for (long long e = 0; e < c->nE; ++e) f[e] = st->element_flag[e] != 0 ? 1 : 0;
        HIPCHK(hipMemcpyAsync(c->d_flag, f.data(), c->nE * sizeof(int), hipMemcpyHostToDevice, s));
        // deleted before the upload: step unknown (-1), never reported by hakai_deleted, but the
        // faces its deletion exposed are live for contact
        std::vector<int> ds((size_t)c->nE);
        for (long long e = 0; e < c->nE; ++e) ds[e] = f[e] ? 0 : -1;
        HIPCHK(hipMemcpyAsync(c->d_del_step, ds.data(), c->nE * sizeof(int), hipMemcpyHostToDevice, s));
        HIPCHK(hipMemsetAsync(c->d_del_step + c->nEp, 0, 2 * sizeof(int), s));  // dump + last-deletion slots
        HIPCHK(hipStreamSynchronize(s));
        // fe of elements uploaded as deleted must not contribute
        bool any = false;
        for (long long e = 0; e < c->nE; ++e) any |= !f[e];
        if (any && !st->Qe) {
            std::vector<double> qe(24 * (size_t)c->nE);
            int r = fe_download_qe(c, qe.data());
            if (r) return r;
            for (long long e = 0; e < c->nE; ++e)
                if (!f[e]) std::fill(qe.begin() + 24 * e, qe.begin() + 24 * (e + 1), 0.0);
            if ((r = fe_upload_qe(c, qe.data()))) return r;
        }
    }
    if (st->Qe) {
        int r = fe_upload_qe(c, st->Qe);
        if (r) return r;
    }
    HIPCHK(hipMemsetAsync(c->d_poison, 0, 2 * sizeof(int), s));
    HIPCHK(hipStreamSynchronize(s));
    c->steps_done = 0;
    c->fe_ok = c->triax_ok = true;
    hkc::comm_reset(c);
    c->state_ok = true;
    if (c->contact) {
        if (int r = hkc::contact_state_reset(c, c->h_velo0.empty() ? nullptr : c->h_velo0.data())) return r;
        HIPCHK(hipStreamSynchronize(s));
    }
    return 0;
}

int hakai_download_state(hakai_ctx* c, hakai_state_t* st) {
    if (!c || !st) return fail(HAKAI_ERR_ARG, "null");
    if (!c->state_ok) return fail(HAKAI_ERR_STATE, "download_state without state");
    if (st->Qe && !c->fe_ok)
        return fail(HAKAI_ERR_STATE, "download_state: Qe is not available after a call whose last steps a contact "
                    "overflow skipped (owner-computed assembly keeps node sums only); Q is -- or step once more");
    if (st->integ_triax_stress && !c->triax_ok)
        return fail(HAKAI_ERR_STATE, "download_state: integ_triax_stress is not available after a call whose last "
                    "steps a contact overflow skipped (it is stored on a call's last step); step once more");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const size_t fn = 3 * (size_t)c->nN, nGP = 8 * (size_t)c->nE;
    HIPCHK(hipStreamSynchronize(s));
    if (st->disp) HIPCHK(hipMemcpyAsync(st->disp, c->d_u[c->cur], fn * sizeof(double), hipMemcpyDeviceToHost, s));
    if (st->disp_pre)
        HIPCHK(hipMemcpyAsync(st->disp_pre, c->d_u[1 - c->cur], fn * sizeof(double), hipMemcpyDeviceToHost, s));
    if (st->velo) {
        if (c->steps_done == 0) {
            std::memcpy(st->velo, c->h_velo0.data(), fn * sizeof(double));
        } else {  // velo = d_disp / d_time with d_disp = disp_new - disp (v2/HAKAI_j.jl:625-628)
            std::vector<double> a(fn), b(fn);
            HIPCHK(hipMemcpyAsync(a.data(), c->d_u[c->cur], fn * sizeof(double), hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(b.data(), c->d_u[1 - c->cur], fn * sizeof(double), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            for (size_t i = 0; i < fn; ++i) {
                const double dd = a[i] - b[i];
                st->velo[i] = dd / c->last_dt;
            }
        }
    }
    if (st->Q) {
        if (c->q_from_buf) {
            HIPCHK(hipMemcpyAsync(st->Q, c->d_qbuf, fn * sizeof(double), hipMemcpyDeviceToHost, s));
        } else {
            double* tmp = nullptr;
            HIPCHK(dalloc(&tmp, fn));
            if (c->own_valid)  // the last element step's owner-computed sums (fe may be stale)
                HIPCHK(hk::launch_own_q(c->d_own_q, c->d_own_rp, c->d_own_ridx, c->d_own_rows, tmp, c->nN, s));
            else
                HIPCHK(hk::launch_gather_q(c->d_inc_ptr, c->d_inc, c->d_fe, tmp, c->nN, s));
            HIPCHK(hipMemcpyAsync(st->Q, tmp, fn * sizeof(double), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            dfree(tmp);
        }
    }
    if (st->integ_stress || st->integ_strain) {
        double* tmp = nullptr;
        HIPCHK(dalloc(&tmp, 6 * nGP));
        if (st->integ_stress) {
            HIPCHK(hk::launch_soa_to_aos6(c->d_stress, tmp, (long long)nGP, c->ld, s));
            HIPCHK(hipMemcpyAsync(st->integ_stress, tmp, 6 * nGP * sizeof(double), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        if (st->integ_strain) {
            HIPCHK(hk::launch_soa_to_aos6(c->d_strain, tmp, (long long)nGP, c->ld, s));
            HIPCHK(hipMemcpyAsync(st->integ_strain, tmp, 6 * nGP * sizeof(double), hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        dfree(tmp);
    }
    if (st->integ_yield_stress)
        HIPCHK(hipMemcpyAsync(st->integ_yield_stress, c->d_yield, nGP * sizeof(double), hipMemcpyDeviceToHost, s));
    if (st->integ_eq_plastic_strain)
        HIPCHK(hipMemcpyAsync(st->integ_eq_plastic_strain, c->d_eqps, nGP * sizeof(double), hipMemcpyDeviceToHost, s));
    if (st->integ_triax_stress)
        HIPCHK(hipMemcpyAsync(st->integ_triax_stress, c->d_triax, nGP * sizeof(double), hipMemcpyDeviceToHost, s));
    if (st->element_flag) {
        std::vector<int> f((size_t)c->nE);
        HIPCHK(hipMemcpyAsync(f.data(), c->d_flag, c->nE * sizeof(int), hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        for (long long e = 0; e < c->nE; ++e) st->element_flag[e] = (f[e] == 1) ? 1 : 0;
    }
    if (st->Qe) {
        int r = fe_download_qe(c, st->Qe);
        if (r) return r;
    }
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

// ---------------------------------------------------------------------------------------------
// Owner-computed assembly (tuning "own_assembly"). Block lb of the persistent element kernel walks
// a SCHEDULE: the batches at positions [bstart[lb], bstart[lb+1]) of seq, ascending in batch id.
// A node's incidences, in ascending element order (the reference's serial sum,
// v2/HAKAI_j.jl:668-675), start with a run held by one block (the head segment). That block sums
// the run in an LDS slot, starting from 0.0 exactly like the nodal gather, and stores the result
// into own_q[n] (the whole Q when the run is all of them). Every later contribution is copied
// unchanged to its own row, rows of a node consecutive in element order, and the nodal kernel
// forms ((own_q[n] + row) + row) ... -- the same additions in the same order as the gather of fe,
// so the result is bit-identical whatever the schedule. Rows are numbered by super-batch (an
// export entry carries up to 4 contributions of any nodes to consecutive rows); own_ridx lists
// each node's rows in element order. One 16-B entry per node segment piece (or exported
// contribution) per super-batch of S = 2 schedule positions (1 when 2 would need more than 512
// entries), one or two per thread (layout: hakai_kernels.hip own_pass). Slots are allocated per
// block over the super-batches a sum is open; a schedule needing more than own_slot_cap open sums in
// one block, or a node with > 8 incidences, does not use the mode.
//
// Schedules (own_use picks the cheapest that fits):
//  * contiguous: block lb holds batches [lb*nb/G, (lb+1)*nb/G) -- a slender section (C3) keeps all
//    of a node layer's sums open in one block;
//  * banded: on a structured region (element ids x-fastest: the +y neighbour is id+nx, the +z one
//    id+L) a wide section (C4's 200x200 plate, C5's 100x100 bar) would keep one whole node layer
//    open (10-40 k sums > 1024 slots), so most contributions became rows. The banded schedule
//    splits each layer into bands of R element rows and gives each block one band over a run of
//    layers: a node's 8 incidences then fall in one block unless it sits on a band or run edge.
// ---------------------------------------------------------------------------------------------
static constexpr int kOwnExpRowsHost = 4;   // = kOwnExpRows: contributions per exported entry
enum { kOwnInitH = 1, kOwnFinH = 2, kOwnExpH = 4, kOwnNopH = 8 };

struct OwnSched {
    int epb = 32;                  // elements per batch: 32 (block units) or 8 (wave units)
    std::vector<int> seq;          // [nb] batch at each position
    std::vector<long long> bstart; // [G+1]
    bool banded = false;
};

struct OwnPlan {
    int S = 2;
    std::vector<int> off, list, rp, ridx;
    long long rows = 0, ne = 0;
    int max_slots = 1;
    long long round2 = 0;  // summing passes with more than one entry per thread
    // per-step bytes the lists add beyond the element/nodal kernels' own (entries read, rows
    // written and read back, row indices): what own_use compares between schedules
    double cost() const { return 16.0 * (double)ne + 52.0 * (double)rows; }
};

static OwnSched own_contiguous(long long nb, long long G, int epb) {
    OwnSched sc;
    sc.epb = epb;
    sc.seq.resize(nb);
    for (long long b = 0; b < nb; ++b) sc.seq[b] = (int)b;
    sc.bstart.resize(G + 1);
    for (long long lb = 0; lb <= G; ++lb) sc.bstart[lb] = lb * nb / G;
    return sc;
}

// Lattice strides of structured regions: element e's (nx, L) from a node whose 8 incidences start
// with e, {e, e+1, e+nx, e+nx+1, e+L, e+L+1, e+L+nx, e+L+nx+1}; elements without such a node (the
// last of a row, layer or region) take the previous element's. Regions = runs of equal strides.
// Returns false when the mesh shows no such lattice.
static bool lattice_strides(const hakai_ctx* c, std::vector<int>& nx, std::vector<int>& L) {
    const long long nE = c->nE;
    nx.assign(nE, -1);
    L.assign(nE, -1);
    long long found = 0;
    for (long long e = 0; e < nE; ++e) {
        for (int k = 0; k < 8; ++k) {
            const int n = c->h_conn[8 * e + k];
            const int j0 = c->h_ptr[n];
            if (c->h_ptr[n + 1] - j0 != 8 || c->h_inc0[j0] / 8 != e) continue;
            long long q[8];
            for (int i = 0; i < 8; ++i) q[i] = c->h_inc0[j0 + i] / 8 - e;
            const long long a = q[2], l = q[4];
            if (q[1] == 1 && a > 1 && q[3] == a + 1 && l > a + 1 && q[5] == l + 1 && q[6] == l + a &&
                q[7] == l + a + 1 && l % a == 0 && l < (1LL << 30)) {
                nx[e] = (int)a;
                L[e] = (int)l;
                ++found;
                break;
            }
        }
    }
    if (found * 2 < nE) return false;
    long long first = -1;
    for (long long e = 0; e < nE; ++e)
        if (nx[e] > 0) {
            first = e;
            break;
        }
    for (long long e = 0; e < nE; ++e) {
        if (nx[e] > 0) continue;
        const long long src = e < first ? first : e - 1;
        nx[e] = nx[src];
        L[e] = L[src];
    }
    return true;
}

// Banded schedule: each batch goes to the band of its first element, (region, row / R); a band's
// batches (ascending) are cut into runs, about G * (band batches) / nb of them per band.
// Band height R per region: a band of R element rows keeps up to about R + 1 node rows of sums
// open in its block -- the R - 1 interior rows of the node layer below, closing row by row while the
// layer above opens, plus what a super-batch holds (measured with tools/own_plan_check: 1071 slots
// at R = 4 on a 200-wide section, 1264 at R = 5) -- so R <= slots * 15/16 / (nx + 1) - 1. Within
// that, the exported rows per node are about 6/R at band edges plus 4 G R / (layers * rows) at run
// edges, least at R = sqrt(1.5 layers rows / G_region).
static bool own_banded(const hakai_ctx* c, long long G, const std::vector<int>& nx, const std::vector<int>& L,
                       int shrink, int epb, int slot_cap, OwnSched& sc) {
    const long long nb = c->nEp / epb, nE = c->nE;
    sc.epb = epb;
    // regions: contiguous id ranges of equal strides
    std::vector<long long> rstart{0};
    for (long long x = 1; x < nE; ++x)
        if (nx[x] != nx[x - 1] || L[x] != L[x - 1]) rstart.push_back(x);
    rstart.push_back(nE);
    std::vector<long long> Rreg(rstart.size() - 1);
    for (size_t r = 0; r + 1 < rstart.size(); ++r) {
        const long long e0 = rstart[r], ne = rstart[r + 1] - e0;
        const long long rows = L[e0] / nx[e0], layers = std::max<long long>(1, ne / L[e0]);
        const double Gr = std::max(1.0, (double)G * (double)ne / (double)nE);
        const long long Rcap = (slot_cap - slot_cap / 16) / (nx[e0] + 1) - 1;
        const long long Ropt = (long long)std::llround(std::sqrt(1.5 * (double)layers * (double)rows / Gr));
        const long long Rwant = c->own_band_rows > 0 ? (long long)c->own_band_rows : std::max<long long>(Ropt, 1);
        Rreg[r] = std::max<long long>(1, std::min(Rcap, Rwant) - shrink);
    }
    std::vector<long long> key(nb);
    bool any_split = false;
    size_t region = 0;
    for (long long b = 0; b < nb; ++b) {
        const long long e = std::min(epb * b, nE - 1);
        while (e >= rstart[region + 1]) ++region;
        const long long rows = L[e] / nx[e];
        long long R = Rreg[region];
        if (R >= rows) R = rows;
        else any_split = true;
        const long long row = ((e - rstart[region]) % L[e]) / nx[e];
        key[b] = ((long long)region << 32) | (row / R);
    }
    if (!any_split) return false;  // one band per layer everywhere: the contiguous schedule
    std::vector<int> order(nb);
    for (long long b = 0; b < nb; ++b) order[b] = (int)b;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return key[x] < key[y]; });
    // bands: [p, q) ranges of the sorted order; runs per band apportioned to exactly G blocks in
    // total (largest remainders, at least one per band): more blocks than the persistent grid would
    // run in a second wave (a whole extra block time)
    std::vector<std::pair<long long, long long>> bands;
    for (long long p = 0; p < nb;) {
        long long q = p;
        while (q < nb && key[order[q]] == key[order[p]]) ++q;
        bands.emplace_back(p, q);
        p = q;
    }
    const long long nbands = (long long)bands.size();
    if (nbands > G) return false;
    std::vector<long long> runs(nbands);
    std::vector<std::pair<double, long long>> rem;
    long long used = 0;
    for (long long i = 0; i < nbands; ++i) {
        const long long m = bands[i].second - bands[i].first;
        const double want = (double)G * (double)m / (double)nb;
        runs[i] = std::max<long long>(1, std::min<long long>(m, (long long)want));
        used += runs[i];
        rem.emplace_back(want - (double)runs[i], i);
    }
    std::sort(rem.begin(), rem.end(), [](const std::pair<double, long long>& x, const std::pair<double, long long>& y) {
        return x.first > y.first || (x.first == y.first && x.second < y.second);
    });
    for (size_t r = 0; used < G && r < rem.size(); ++r) {
        const long long i = rem[r].second;
        if (runs[i] < bands[i].second - bands[i].first) {
            ++runs[i];
            ++used;
        }
    }
    for (long long i = 0; used > G && i < nbands; ++i)  // (the minimum of one run per band overshot)
        while (runs[i] > 1 && used > G) {
            --runs[i];
            --used;
        }
    sc.seq = order;
    sc.bstart.assign(1, 0);
    for (long long i = 0; i < nbands; ++i) {
        const long long p = bands[i].first, m = bands[i].second - p;
        for (long long r = 1; r <= runs[i]; ++r) sc.bstart.push_back(p + r * m / runs[i]);
    }
    sc.banded = true;
    return true;
}

static bool own_plan(const hakai_ctx* c, const OwnSched& sc, int S, int slot_cap, OwnPlan& pl) {
    const int epb = sc.epb, bs = 8 * epb;  // elements per batch, threads per block
    const long long nb = c->nEp / epb, nN = c->nN;
    const long long G = (long long)sc.bstart.size() - 1;
    if (G <= 0 || c->max_inc > 8 || c->h_ptr.size() != (size_t)nN + 1) return false;
    pl.S = S;
    struct Ent { int target, slot, flags, n; int lanes[8]; int inc[4]; };  // inc: an EXP entry's incidences
    // pos_of[b]: schedule position of batch b; block_of[b]; sb_pos[b] = position of the first batch
    // of b's super-batch (runs of S positions from each block's first), which indexes the lists
    std::vector<int> pos_of(nb), block_of(nb);
    std::vector<long long> sb_pos(nb);
    for (long long lb = 0; lb < G; ++lb)
        for (long long p = sc.bstart[lb]; p < sc.bstart[lb + 1]; ++p) {
            const int b = sc.seq[p];
            if (p > sc.bstart[lb] && b <= sc.seq[p - 1]) return false;  // ascending within a block
            pos_of[b] = (int)p;
            block_of[b] = (int)lb;
            sb_pos[b] = sc.bstart[lb] + (p - sc.bstart[lb]) / S * S;
        }
    std::vector<std::vector<Ent>> per(nb);
    std::vector<int> rp(nN + 1, 0);
    long long rows = 0;
    // open-sum intervals per block in super-batch units: (first, last, entry refs to patch the slot)
    struct Seg { long long s0, s1; std::vector<std::pair<long long, int>> refs; };
    std::vector<std::vector<Seg>> segs(G);
    auto batch_of = [&](int j) { return (long long)(c->h_inc0[j] / 8) / epb; };
    // LDS lane of incidence j within its super-batch: (position - super-batch position) * epb +
    // element within the batch, times 8, + local node
    auto lane_of = [&](int j) {
        const long long e = c->h_inc0[j] / 8;
        const long long b = e / epb;
        return (int)(((pos_of[b] - sb_pos[b]) * epb + e % epb) * 8 + c->h_inc0[j] % 8);
    };
    // contributions of later segments: (super-batch, incidence index j); their rows are numbered
    // in super-batch order so that one entry exports up to 4 of them (any nodes) to consecutive rows
    std::vector<std::pair<long long, int>> exports;
    // multi-GPU: the nodes shared with rank-1 send their contributions one by one (hakai_comm.cpp
    // k_pack_own), so all of them are rows
    std::vector<char> all_rows(nN, 0);
    if (const std::vector<int>* dn = hkc::comm_dn_nodes(c))
        for (int n : *dn) all_rows[n] = 1;
    for (long long n = 0; n < nN; ++n) {
        const int j0 = c->h_ptr[n], j1 = c->h_ptr[n + 1];
        if (j0 == j1) continue;
        if (all_rows[n]) {
            for (int j = j0; j < j1; ++j) exports.emplace_back(sb_pos[batch_of(j)], j);
            continue;
        }
        const int hb = block_of[batch_of(j0)];
        int j = j0;
        Seg sg;
        sg.s0 = -1;
        while (j < j1 && block_of[batch_of(j)] == hb) {  // the head segment, super-batch by super-batch
            const long long sb = sb_pos[batch_of(j)];
            Ent en{(int)n, 0, 0, 0, {0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0}};
            while (j < j1 && sb_pos[batch_of(j)] == sb) {
                if (en.n == 8) return false;
                en.lanes[en.n++] = lane_of(j);
                ++j;
            }
            if (sg.s0 < 0) {
                sg.s0 = sb;
                en.flags |= kOwnInitH;
            }
            sg.s1 = sb;
            per[sb].push_back(en);
            sg.refs.emplace_back(sb, (int)per[sb].size() - 1);
        }
        per[sg.s1][sg.refs.back().second].flags |= kOwnFinH;
        if (sg.s1 > sg.s0) segs[hb].push_back(std::move(sg));
        for (; j < j1; ++j) exports.emplace_back(sb_pos[batch_of(j)], j);
    }
    // rows: grouped by super-batch (stable: node order, then element order within a node)
    std::stable_sort(exports.begin(), exports.end(),
                     [](const std::pair<long long, int>& x, const std::pair<long long, int>& y) { return x.first < y.first; });
    std::vector<int> row_of_inc(c->h_inc0.size(), -1);
    for (size_t q = 0; q < exports.size();) {
        const long long sb = exports[q].first;
        Ent en{0, 0, kOwnExpH, 0, {0, 0, 0, 0, 0, 0, 0, 0}, {0, 0, 0, 0}};
        while (q < exports.size() && exports[q].first == sb && en.n < kOwnExpRowsHost) {
            const int j = exports[q].second;
            en.inc[en.n] = j;
            en.lanes[en.n++] = lane_of(j);
            ++q;
        }
        per[sb].push_back(en);
    }
    // Row numbers, coalesced by wave: the EXP entries of a super-batch that one wave of the pass
    // takes (list positions in one 64-aligned window, a contiguous run: they follow the node
    // entries) form a group of g entries with m <= 4 g contributions in export order (node, then
    // element). Contribution q of the group goes to row base + q, dealt to entry q mod g as its
    // (q / g)-th: so the wave's k-th stores cover g consecutive rows, and a node's rows stay
    // consecutive for the nodal kernel. An entry's target is base + i, its stride g rides in the
    // unused slot field.
    for (long long b = 0; b < nb; ++b) {
        std::vector<Ent>& v = per[b];
        for (size_t p = 0; p < v.size();) {
            if (!(v[p].flags & kOwnExpH)) {
                ++p;
                continue;
            }
            size_t p1 = p;
            while (p1 < v.size() && (v[p1].flags & kOwnExpH) && p1 / 64 == p / 64) ++p1;
            const int g = (int)(p1 - p);
            std::vector<std::pair<int, int>> cs;  // (incidence, lane) in export order
            for (size_t i = p; i < p1; ++i)
                for (int k = 0; k < v[i].n; ++k) cs.emplace_back(v[i].inc[k], v[i].lanes[k]);
            const int m = (int)cs.size();
            for (int i = 0; i < g; ++i) {
                Ent& en = v[p + (size_t)i];
                en.target = (int)(rows + i);
                en.slot = g;
                en.n = 0;
                for (int q = i; q < m; q += g) {
                    en.inc[en.n] = cs[(size_t)q].first;
                    en.lanes[en.n++] = cs[(size_t)q].second;
                    row_of_inc[cs[(size_t)q].first] = (int)(rows + q);
                }
            }
            rows += m;
            p = p1;
        }
    }
    // per node: its rows in element order (CSR rp / ridx)
    std::vector<int>& ridx = pl.ridx;
    ridx.clear();
    ridx.reserve(exports.size());
    for (long long n = 0; n < nN; ++n) {
        rp[n] = (int)ridx.size();
        for (int j = c->h_ptr[n]; j < c->h_ptr[n + 1]; ++j)
            if (row_of_inc[j] >= 0) ridx.push_back(row_of_inc[j]);
    }
    rp[nN] = (int)ridx.size();
    if (rows > (1LL << 31) - 1) return false;
    // slots: a sum open over super-batches [s0, s1] holds its slot through s1; reuse strictly after
    int max_slots = 1;
    for (long long lb = 0; lb < G; ++lb) {
        auto& v = segs[lb];
        std::sort(v.begin(), v.end(), [](const Seg& x, const Seg& y) { return x.s0 < y.s0; });
        std::vector<std::pair<long long, int>> busy;  // (s1, slot) min-heap
        std::vector<int> free_slots;
        int next = 0;
        auto cmp = [](const std::pair<long long, int>& x, const std::pair<long long, int>& y) { return x.first > y.first; };
        for (auto& sg : v) {
            while (!busy.empty() && busy.front().first < sg.s0) {
                free_slots.push_back(busy.front().second);
                std::pop_heap(busy.begin(), busy.end(), cmp);
                busy.pop_back();
            }
            int slot;
            if (!free_slots.empty()) {
                slot = free_slots.back();
                free_slots.pop_back();
            } else {
                slot = next++;
            }
            if (slot >= slot_cap) return false;
            max_slots = std::max(max_slots, slot + 1);
            for (auto& r : sg.refs) per[r.first][r.second].slot = slot;
            busy.emplace_back(sg.s1, slot);
            std::push_heap(busy.begin(), busy.end(), cmp);
        }
    }
    std::vector<int>& off = pl.off;
    off.assign(nb + 1, 0);
    for (long long b = 0; b < nb; ++b) {
        if (per[b].size() > 2 * (size_t)bs) return false;  // two entries per thread at most (own_pass)
        pl.round2 += per[b].size() > (size_t)bs ? 1 : 0;
        off[b + 1] = off[b] + (int)per[b].size();
    }
    const long long ne = off[nb];
    std::vector<int>& list = pl.list;
    list.assign(4 * (size_t)(ne + 1), 0);
    for (long long b = 0; b < nb; ++b)
        for (size_t i = 0; i < per[b].size(); ++i) {
            const Ent& en = per[b][i];
            unsigned long long lo = 0;
            for (int q = 0; q < 7; ++q) lo |= (unsigned long long)en.lanes[q] << (9 * q);
            int* w = &list[4 * ((size_t)off[b] + i)];
            w[0] = en.target;
            w[1] = (int)(((unsigned)en.slot & 1023u) | (unsigned)en.flags << 10 | (unsigned)en.n << 14 |
                         (unsigned)en.lanes[7] << 18 | ((unsigned)en.slot & 1024u) << 18);
            w[2] = (int)(unsigned)(lo & 0xffffffffu);
            w[3] = (int)(unsigned)(lo >> 32);
        }
    int* nop = &list[4 * (size_t)ne];  // padding entry: reads lane 0, stores to the dump line
    nop[1] = kOwnNopH << 10;
    pl.rp = std::move(rp);
    pl.rows = rows;
    pl.ne = ne;
    pl.max_slots = max_slots;
    return true;
}

static bool own_upload(hakai_ctx* c, const OwnSched& sc, const OwnPlan& pl) {
    hkc::own_free(c);
    const long long nN = c->nN, G = (long long)sc.bstart.size() - 1;
    std::vector<int> bst(sc.bstart.begin(), sc.bstart.end());
    hipStream_t s = c->stream;
    auto up = [&](int** d, const std::vector<int>& h) -> hipError_t {
        hipError_t e = dalloc(d, std::max<size_t>(h.size(), 1));
        if (e == hipSuccess && !h.empty()) e = hipMemcpyAsync(*d, h.data(), h.size() * sizeof(int), hipMemcpyHostToDevice, s);
        return e;
    };
    if (up(&c->d_own_off, pl.off) || up(&c->d_own_seq, sc.seq) || up(&c->d_own_bstart, bst) ||
        up(&c->d_own_list, pl.list) || up(&c->d_own_rp, pl.rp) || up(&c->d_own_ridx, pl.ridx) ||
        dalloc(&c->d_own_q, 3 * (size_t)nN) || dalloc(&c->d_own_rows, 3 * (size_t)std::max(pl.rows, 1LL)) ||
        dalloc(&c->d_own_dump, 8 * (size_t)G) ||
        hipMemsetAsync(c->d_own_q, 0, 3 * (size_t)nN * sizeof(double), s) ||  // nodes without elements
        hipStreamSynchronize(s)) {
        hkc::own_free(c);
        return false;
    }
    c->own_nop = (int)pl.ne;
    c->own_slots = pl.max_slots;
    c->own_rows = pl.rows;
    c->own_entries = pl.ne;
    c->own_built_g = G;
    c->own_s = pl.S;
    c->own_round2 = pl.round2;
    c->own_banded = sc.banded ? 1 : 0;
    return true;
}

// Grid of the persistent kernel for this context (0: the one-batch kernel runs).
static long long own_grid(const hakai_ctx* c) {
    const long long nb = c->nEp / 32;
    const bool pipe = nb >= (long long)c->pipe_min * c->pipe_blocks && c->pipe_blocks > 0;
    return pipe ? std::min<long long>(nb, c->pipe_blocks) : 0;
}

// This step's element update uses owner-computed assembly (builds the lists on first use). The
// grid is the persistent kernel's, or 8x that (blocks then run in waves) when the default ranges
// span so much of a wide cross-section that too many sums stay open in a block.
// Owner assembly stops being used while the previous element step's forces exist only as its
// node sums (a tuning change, a list rebuild): hand the next nodal update Q through the uploaded-Q
// buffer, the same bits (k_own_q = k_nodal's own additions). Multi-GPU ranks cannot: their next
// interface fix needs the per-contribution rows.
static int own_materialize(hakai_ctx* c) {
    if (!c->own_valid) return 0;
    if (c->comm)
        return fail(HAKAI_ERR_STATE, "owner-computed assembly cannot be switched off or rebuilt on a multi-GPU rank "
                    "mid-run: upload or reset the state first");
    HIPCHK(hk::launch_own_q(c->d_own_q, c->d_own_rp, c->d_own_ridx, c->d_own_rows, c->d_qbuf, c->nN, c->stream));
    c->q_from_buf = true;
    c->own_valid = false;
    return 0;
}

// Candidate schedules, cheapest plan wins (OwnPlan::cost): contiguous at the persistent grid G0,
// banded at about G0 blocks (when the mesh has a structured wide section), and, if neither fits,
// contiguous at 8 G0 (finer ranges keep fewer sums open; the blocks run in waves). Super-batches
// of 2 batches where they fit 512 entries, else 1. `only` (the CPU replay harness,
// tools/own_plan_check.cpp): 0 every schedule, 1 contiguous only, 2 banded only.
static bool own_choose(hakai_ctx* c, long long G0, OwnSched& best_sc, OwnPlan& best, int only = 0) {
    const int epb = 32;
    const long long nb = c->nEp / epb;
    // slots per block: what two blocks per CU leave next to the kernel's own LDS (the wider
    // passes of S = 2 leave less); row bands are sized for S = 2
    auto cap_of = [&](int S) { return hk::own_slot_cap(c->elem_exact != 0, S, c->nmat); };
    const int cap = cap_of(2);
    bool have = false;
    auto consider = [&](const OwnSched& sc) {
        for (int S : {2, 1}) {
            if (c->own_pass_batches > 0 && S != c->own_pass_batches) continue;
            OwnPlan pl;
            if (!own_plan(c, sc, S, cap_of(S), pl)) continue;
            if (!have || pl.cost() < best.cost()) {
                best = std::move(pl);
                best_sc = sc;
                have = true;
            }
            return true;  // S = 2 fits: S = 1 only adds passes
        }
        return false;
    };
    if (only != 2) consider(own_contiguous(nb, G0, epb));
    if (only != 1) {
        std::vector<int> nx, L;
        if (lattice_strides(c, nx, L)) {
            OwnSched sc;
            for (int shrink : {0, 1, 2, 4})  // the widest bands whose open sums fit a block's slots
                if (own_banded(c, G0, nx, L, shrink, epb, cap, sc) && consider(sc)) break;
        }
    }
    if (!have && only != 2 && 8 * G0 <= nb) consider(own_contiguous(nb, 8 * G0, epb));
    return have;
}

static bool own_use(hakai_ctx* c) {
    if (!c->own_assembly || c->nmat > hk::kMaxLdsMats || c->nE <= 0)
        return false;
    const long long G0 = own_grid(c);
    if (G0 <= 0) return false;
    bool ok = c->own_built_g > 0;
    if (c->own_for_g0 != G0) {  // not yet built (or found not to fit) for this grid
        if (c->own_valid && own_materialize(c)) return false;  // (multi-GPU: step_once reports it)
        OwnSched sc;
        OwnPlan pl;
        ok = own_choose(c, G0, sc, pl) && own_upload(c, sc, pl);
        if (!ok) {
            hkc::own_free(c);
            c->own_built_g = -2;
        }
        c->own_for_g0 = G0;
    }
    // The reference-order kernel's waves drift apart within a batch more than the fused kernel's, so
    // its block waits at the pass barrier for its slowest wave; passes that load a second entry
    // inside that barrier region (wide cross-sections) make the wait long, and there the fe path is
    // faster for this kernel (C5 slab 1.12 against 1.41 ms per step, C4 2.46 against 3.25,
    // profiles/r03_wave_units_sweep.log). own_assembly 2 uses the owner sums anyway (tests); a
    // multi-GPU rank whose owner sums are live keeps them (its interface fix needs the rows).
    if (ok && c->elem_exact && c->own_round2 > 0 && c->own_assembly == 1 && !(c->comm && c->own_valid))
        return false;
    return ok;
}

// One explicit step (the loop body :497-764). With c->g_trd set (graph capture) the kernels take
// the step number from the device counter and the element kernel advances it. Phase bits: the
// contact search parts A1, A2, A3 (hkc::contact_phase; one GPU: all of it in A1) and the rest
// (contact phase B, nodal, BCs, element, exchange). An in-process group with multi-GPU contact runs
// each part on every rank before the next (hakai_step_group).
enum { kPhaseA1 = 1, kPhaseRest = 2, kPhaseA2 = 4, kPhaseA3 = 8, kPhaseAll = 15 };
static int step_once(hakai_ctx* c, double t, double d_time, bool last, int phase = kPhaseAll) {
    hipStream_t s = c->stream;
    EventPair ep;
    if (c->contact) {  // contact force into external_force (:500-560), search parts
        const int part_bit[3] = {kPhaseA1, kPhaseA2, kPhaseA3};
        for (int part = 1; part <= 3; ++part) {
            if (!(phase & part_bit[part - 1]) || (part > 1 && !hkc::contact_multi(c))) continue;
            hkc::prof_begin(c, HAKAI_K_CONTACT, &ep);
            const int rc = hkc::contact_phase(c, part, t, d_time);
            hkc::prof_end(c, &ep);
            if (rc) return rc;
        }
    }
    if (!(phase & kPhaseRest)) return 0;
    const int par = c->cur;  // graph mode: this step reads counter slot 1-par, writes slot par
    // nodal update (:562-567), Q from the previous step's element forces (:668-675)
    hk::NodalArgs na;
    na.u = c->d_u[c->cur];
    na.u_pre_out = c->d_u[1 - c->cur];
    na.mass = c->d_mass;
    na.inc_ptr = c->d_inc_ptr;
    na.inc = c->d_inc;
    na.inc8 = c->d_inc8;
    na.fe = c->d_fe;
    // owner-computed assembly: Q from the previous element step's sums (else the fe gather)
    const bool own = own_use(c);
    if (c->own_valid && !own) {  // switched off (or the lists could not be rebuilt)
        if (int r = own_materialize(c)) return r;
    }
    na.qbuf = c->q_from_buf ? c->d_qbuf : nullptr;
    na.fext = nullptr;
    na.nN = c->nN;
    na.dt = d_time;
    na.bc_of_node = nullptr;
    const bool own_q = c->own_valid && !na.qbuf;
    na.own_q = own_q ? c->d_own_q : nullptr;
    na.own_rp = own_q ? c->d_own_rp : nullptr;
    na.own_rows = own_q ? c->d_own_rows : nullptr;
    na.own_ridx = own_q ? c->d_own_ridx : nullptr;
    hk::BCArgs ba;
    ba.dof = c->d_bc_dof;
    ba.grp = c->d_bc_grp;
    ba.val = c->d_bc_val;
    ba.n = c->nbc;
    ba.amp_n = c->d_amp_n;
    ba.amp_off = c->d_amp_off;
    ba.amp_t = c->d_amp_t;
    ba.amp_v = c->d_amp_v;
    ba.out = c->d_u[1 - c->cur];
    ba.ct = t * d_time;
    ba.t_rd = c->g_trd;
    ba.dt = d_time;
    ba.poison = c->d_poison;
    na.poison = c->d_poison;
    // one GPU, small mesh: the nodal kernel applies the BCs (multi-GPU redoes interface nodes
    // after the nodal kernel, so the BCs must come after that)
    // (fuse_bc 2: at any size; large meshes measured slower with the fe gather, see kFuseBcMaxNodes)
    const bool fuse_bc = c->nbc > 0 && c->d_bc_of_node && c->fuse_bc && !c->comm &&
                         (c->nN <= kFuseBcMaxNodes || c->fuse_bc == 2);
    if (fuse_bc) {
        na.bc_of_node = c->d_bc_of_node;
        na.bc = ba;
    }
    int rc = 0;
    if (c->contact) {  // multi-GPU search: event exchange and force sums
        if (hkc::contact_multi(c)) {
            hkc::prof_begin(c, HAKAI_K_CONTACT_SUM, &ep);
            rc = hkc::contact_step_b(c);
            hkc::prof_end(c, &ep);
            if (rc) return rc;
        }
        na.fext = c->d_fext;
    }
    rc = hkc::comm_pre_nodal(c);
    if (rc) return rc;
    hkc::prof_begin(c, HAKAI_K_NODAL, &ep);
    HIPCHK(hk::launch_nodal(na, s));
    hkc::prof_end(c, &ep);
    // multi-GPU: interface nodes are redone with the cross-rank assembled Q
    rc = hkc::comm_post_nodal(c, d_time);
    if (rc) return rc;
    // boundary conditions (:585-617)
    if (c->nbc > 0 && !fuse_bc) {
        hkc::prof_begin(c, HAKAI_K_BC, &ep);
        HIPCHK(hk::launch_bc(ba, s));
        hkc::prof_end(c, &ep);
    }
    c->cur = 1 - c->cur;  // disp <- disp_new, disp_pre <- disp (:626-627)
    c->q_from_buf = false;
    // element update (:662-667) + triaxiality (:677) + ductile deletion (:684-764)
    hk::ElemArgs ea = elem_args(c);
    ea.step_i = (int)t;
    if (own) {
        ea.own = c->own_s;
        ea.own_grid = (int)c->own_built_g;
        ea.own_seq = c->d_own_seq;
        ea.own_bstart = c->d_own_bstart;
        ea.own_off = c->d_own_off;
        ea.own_list = reinterpret_cast<const int4*>(c->d_own_list);
        ea.own_nop = c->own_nop;
        ea.own_slots = c->own_slots;
        ea.own_q = c->d_own_q;
        ea.own_rows = c->d_own_rows;
        ea.own_dump = c->d_own_dump;
    }
    if (c->g_trd) {
        ea.t_rd = c->g_trd;
        ea.t_wr = c->d_tstep + par;
    }
    hkc::prof_begin(c, HAKAI_K_ELEMENT, &ep);
    HIPCHK(hk::launch_element(ea, c->has_ductile, last, s));
    hkc::prof_end(c, &ep);
    c->own_valid = own;
    c->own_steps += own ? 1 : 0;
    c->fe_ok = !own || last;  // owner assembly stores fe on a call's last step only
    c->triax_ok = last;
    rc = hkc::comm_post_element(c, (long long)t);
    if (rc) return rc;
    rc = hkc::contact_post_step(c);
    if (rc) return rc;
    c->steps_done++;
    c->last_dt = d_time;
    return 0;
}

// A run of steps starting at t can come from a graph: same launch sequence every step, nothing
// host-side that depends on the step (no multi-GPU exchange, no profiling events, no uploaded Q),
// and contact in its steady state. The step number comes from a device counter; every pointer
// argument is fixed for a given starting parity (cur), so one graph per parity serves the whole
// run. A failed capture leaves the context's host state advanced: the call returns the error.
static bool graph_eligible(const hakai_ctx* c, double t) {
    // (owner-computed assembly: only once the previous step left its sums, so every captured nodal
    // update reads them)
    return c->graph && !c->comm && !c->prof && !c->q_from_buf && c->nE > 0 && hkc::contact_graph_ok(c, t) &&
           c->own_valid == own_use(const_cast<hakai_ctx*>(c));
}

static int step_graph(hakai_ctx* c, double t, double d_time, int len) {
    hipStream_t s = c->stream;
    const int p0 = c->cur;
    const int gi = len == 2 ? 1 : 0;
    hipGraphExec_t& ge = c->g_exec[gi][p0];
    if (!c->d_tstep) HIPCHK(dalloc(&c->d_tstep, 2));
    if (c->tdev_next != (long long)t) HIPCHK(hk::launch_set_step(c->d_tstep + (1 - p0), t - 1.0, s));
    if (ge && (c->g_epoch[gi][p0] != c->epoch || c->g_dt[gi][p0] != d_time || c->g_len[gi][p0] != len)) {
        HIPCHK(hipStreamSynchronize(s));
        (void)hipGraphExecDestroy(ge);
        ge = nullptr;
    }
    if (!ge) {
        // capture the steps; their host-side state changes happen here, as in stream mode
        hipGraph_t g = nullptr;
        HIPCHK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        int rc = 0;
        for (int k = 0; k < len && !rc; ++k) {
            c->g_trd = c->d_tstep + (1 - c->cur);
            rc = step_once(c, t + k, d_time, false);
        }
        c->g_trd = nullptr;
        hipError_t e = hipStreamEndCapture(s, &g);
        if (rc) {
            if (g) (void)hipGraphDestroy(g);
            return rc;
        }
        if (e != hipSuccess) return hip_fail(e, "hipStreamEndCapture (step graph)");
        e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        if (e != hipSuccess) {
            ge = nullptr;
            return hip_fail(e, "hipGraphInstantiate (step graph)");
        }
        c->g_epoch[gi][p0] = c->epoch;
        c->g_dt[gi][p0] = d_time;
        c->g_len[gi][p0] = len;
    } else {  // replay the host-side state changes of the captured steps
        hkc::contact_graph_advance(c, t + len - 1);
        c->q_from_buf = false;
        c->own_steps += c->own_valid ? len : 0;  // captured in the steady state: every step or none
        c->fe_ok = !c->own_valid;                 // (a captured step is never a call's last)
        c->triax_ok = false;
        c->steps_done += len;
        c->last_dt = d_time;
    }
    HIPCHK(hipGraphLaunch(ge, s));
    c->tdev_next = (long long)t + len;
    c->graph_steps += len;
    return 0;
}

// The host's view of a context before a stepping call's first step (after any owner-assembly
// re-plan, which hands the last sums over unchanged): what an overflow on that step rolls back to.
struct CallSnap {
    int cur = 0;
    long long done = 0;
    bool fe_ok = true, triax_ok = true, own_valid = false, q_from_buf = false;
    bool comm_pending = false;  // the interface exchange the call's first nodal update consumes
    int comm_par = 0;
};
static CallSnap call_snap(const hakai_ctx* c) {
    CallSnap s;
    hkc::comm_pending_get(c, &s.comm_pending, &s.comm_par);
    s.cur = c->cur;
    s.done = c->steps_done;
    s.fe_ok = c->fe_ok;
    s.triax_ok = c->triax_ok;
    s.own_valid = c->own_valid;
    s.q_from_buf = c->q_from_buf;
    return s;
}

// End of a stepping call: the contact overflow check. An overflow poisoned step p: the device's
// state-writing kernels of steps p.. were no-ops, so the device holds the state after step p-1;
// bring the host's view back to that step.
static int finish_call(hakai_ctx* c, double t_first, int64_t n_steps, const CallSnap& s0) {
    const int rc = hkc::contact_check(c);
    if (rc && c->contact) {
        int pz[2] = {0, 0};
        HIPCHK(hipMemcpy(pz, c->d_poison, sizeof pz, hipMemcpyDeviceToHost));
        if (pz[0]) {
            c->poison_step = pz[1];
            const long long good = (long long)pz[1] - (long long)t_first;  // steps of this call that ran
            const bool rolled = good >= 0 && good <= n_steps;
            if (rolled) {
                c->cur = (good & 1) ? 1 - s0.cur : s0.cur;
                c->steps_done = s0.done + good;
                if (good == 0) {  // nothing of the call ran: where the Q of the next nodal update is
                    c->fe_ok = s0.fe_ok;
                    c->triax_ok = s0.triax_ok;
                    c->own_valid = s0.own_valid;
                    c->q_from_buf = s0.q_from_buf;
                } else {  // the call's last step (the one that stores fe and triax) did not run
                    c->fe_ok = !c->own_valid;
                    c->triax_ok = false;
                }
                hkc::comm_rollback(c, good > 0, (long long)pz[1] - 1, s0.comm_pending, s0.comm_par);
            }
            hkc::graph_invalidate(c);
            hkc::contact_after_overflow(c, c->steps_done);
            // a poison step outside this call rolled nothing back: never run the call again from it
            if (!rolled) (void)hkc::contact_exchange_retry(c);
            HIPCHK(hipMemset(c->d_poison, 0, 2 * sizeof(int)));
            const std::string msg = hakai_last_error();
            return fail(rc, "%s; step %d was not applied: the state is that after step %d", msg.c_str(), pz[1],
                        pz[1] - 1);
        }
    }
    return rc;
}

static int step_call(hakai_ctx* c, double t_first, int64_t n_steps, double d_time);
static constexpr int kExchangeRetries = 8;

int hakai_step(hakai_ctx* c, double t_first, int64_t n_steps, double d_time) {
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    if (!c->model_ok || !c->state_ok) return fail(HAKAI_ERR_STATE, "step before upload_model/reset_state");
    if (n_steps < 0 || !(d_time > 0)) return fail(HAKAI_ERR_ARG, "step: n_steps=%lld d_time=%g", (long long)n_steps, d_time);
    if (n_steps > 1 && hkc::comm_is_local(c))
        return fail(HAKAI_ERR_ARG, "step: an in-process group is stepped one step per call, rank by rank");
    // a contact rank of an in-process group needs its peers' phases between its own: refused before
    // any work, so its contact state (tsel parity, touched lists, bin headers) stays in step with them
    if (hkc::comm_is_local(c) && hkc::contact_multi(c) && hkc::comm_size(c) > 1)
        return fail(HAKAI_ERR_STATE, "step: rank %d of an in-process group with multi-GPU contact is stepped by "
                    "hakai_step_group only", hkc::comm_rank(c));
    HIPCHK(hipSetDevice(c->device));
    // a step that overflowed a multi-GPU contact exchange runs again once its capacity has grown
    // (every rank takes the same decision from the same gathered counts)
    for (int attempt = 0;; ++attempt) {
        const int rc = step_call(c, t_first, n_steps, d_time);
        if (!rc || attempt >= kExchangeRetries || !hkc::contact_exchange_retry(c)) return rc;
        ++c->exchange_retries;
        n_steps -= (int64_t)(c->poison_step - (long long)t_first);
        t_first = (double)c->poison_step;
    }
}

static int step_call(hakai_ctx* c, double t_first, int64_t n_steps, double d_time) {
    (void)own_use(c);  // owner-assembly lists are built here, never inside a graph capture
    const CallSnap s0 = call_snap(c);
    int64_t it = 0;
    while (it < n_steps) {
        const double t = t_first + (double)it;
        int rc;
        // the call's last step stays in stream mode: it also stores triaxiality for downloads
        // (eligibility of step t implies it for the steps after it: step t clears every one-off
        // condition)
        const int len = (c->graph > 2 && it + c->graph < n_steps) ? c->graph : 2;
        if (c->graph && it + len < n_steps && graph_eligible(c, t)) {
            rc = step_graph(c, t, d_time, len);
            it += len;
        } else {
            rc = step_once(c, t, d_time, it == n_steps - 1);
            c->tdev_next = -1;
            ++it;
        }
        if (rc) return rc;
    }
    return finish_call(c, t_first, n_steps, s0);
}

static int step_group_call(hakai_ctx** ctxs, int32_t n, double t_first, int64_t n_steps, double d_time) {
    std::vector<CallSnap> s0(n);
    for (int r = 0; r < n; ++r) {
        (void)own_use(ctxs[r]);  // (re-plans here, as hakai_step does, not inside the first step)
        s0[r] = call_snap(ctxs[r]);
    }
    // per step: each contact part on every rank before the next part on any, then the rest
    const int phases[4] = {kPhaseA1, kPhaseA2, kPhaseA3, kPhaseRest};
    for (int64_t it = 0; it < n_steps; ++it) {
        const double t = t_first + (double)it;
        const bool last = it == n_steps - 1;
        for (int ph : phases)
            for (int r = 0; r < n; ++r) {
                // group_serial 2: the phase is enqueued behind a fixed sleep (≈0.3 ms), so its kernels
                // run back to back as in a pipelined run, not at the host's enqueue pace
                if (ctxs[0]->group_serial == 2) HIPCHK(hk::launch_hold(96, ctxs[r]->stream));
                if (int rc = step_once(ctxs[r], t, d_time, last, ph)) return rc;
                if (ph == kPhaseRest) ctxs[r]->tdev_next = -1;
                if (ctxs[0]->group_serial) HIPCHK(hipStreamSynchronize(ctxs[r]->stream));
            }
    }
    int first = 0;
    for (int r = 0; r < n; ++r) {
        const int rc = finish_call(ctxs[r], t_first, n_steps, s0[r]);
        if (rc && !first) first = rc;
    }
    return first;
}

int hakai_step_group(hakai_ctx** ctxs, int32_t n, double t_first, int64_t n_steps, double d_time) {
    if (!ctxs || n <= 0) return fail(HAKAI_ERR_ARG, "step_group: no contexts");
    if (n_steps < 0 || !(d_time > 0)) return fail(HAKAI_ERR_ARG, "step_group: n_steps=%lld d_time=%g",
                                                  (long long)n_steps, d_time);
    for (int r = 0; r < n; ++r) {
        hakai_ctx* c = ctxs[r];
        if (!c) return fail(HAKAI_ERR_ARG, "step_group: null context %d", r);
        if (!c->model_ok || !c->state_ok) return fail(HAKAI_ERR_STATE, "step_group: rank %d has no model/state", r);
        if (n > 1 && (!c->comm || hkc::comm_rank(c) != r || hkc::comm_size(c) != n ||
                      hkc::comm_peer_ctx(c, r) != c))
            return fail(HAKAI_ERR_ARG, "step_group: context %d is not rank %d of an in-process group of %d", r, r, n);
        hkc::graph_invalidate(c);
    }
    HIPCHK(hipSetDevice(ctxs[0]->device));
    for (int attempt = 0;; ++attempt) {
        const int rc = step_group_call(ctxs, n, t_first, n_steps, d_time);
        if (!rc || attempt >= kExchangeRetries) return rc;
        bool retry = true;  // (the same on every rank: they read the same headers)
        for (int r = 0; r < n; ++r) retry = hkc::contact_exchange_retry(ctxs[r]) && retry;
        if (!retry) return rc;
        const long long p = ctxs[0]->poison_step;
        for (int r = 1; r < n; ++r)  // every rank read the same headers: the same step, or no retry
            if (ctxs[r]->poison_step != p)
                return fail(rc, "step_group: ranks disagree on the poisoned step (rank 0: %lld, rank %d: %lld)", p, r,
                            ctxs[r]->poison_step);
        for (int r = 0; r < n; ++r) ++ctxs[r]->exchange_retries;
        n_steps -= (int64_t)(p - (long long)t_first);
        t_first = (double)p;
    }
}

int hakai_graph_steps(hakai_ctx* c, int64_t* n) {
    if (!c || !n) return fail(HAKAI_ERR_ARG, "null");
    *n = c->graph_steps;
    return 0;
}

int hakai_stat(hakai_ctx* c, const char* key, int64_t* value) {
    if (!c || !key || !value) return fail(HAKAI_ERR_ARG, "null");
    if (!std::strcmp(key, "graph_steps")) *value = c->graph_steps;
    else if (!std::strcmp(key, "own_steps")) *value = c->own_steps;
    else if (!std::strcmp(key, "exchange_retries")) *value = c->exchange_retries;
    else if (!std::strcmp(key, "own_rows")) *value = c->own_built_g > 0 ? c->own_rows : -1;
    else if (!std::strcmp(key, "own_entries")) *value = c->own_built_g > 0 ? c->own_entries : -1;
    else if (!std::strcmp(key, "own_superbatch")) *value = c->own_built_g > 0 ? c->own_s : 0;
    else if (!std::strcmp(key, "own_round2")) *value = c->own_built_g > 0 ? c->own_round2 : 0;
    else if (!std::strcmp(key, "own_slots")) *value = c->own_built_g > 0 ? c->own_slots : 0;
    else if (!std::strcmp(key, "own_banded")) *value = c->own_built_g > 0 ? c->own_banded : 0;
    else if (!std::strcmp(key, "own_grid")) *value = c->own_built_g > 0 ? c->own_built_g : 0;
    else return fail(HAKAI_ERR_ARG, "unknown stat '%s'", key);
    return 0;
}

int hakai_sync(hakai_ctx* c) {
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    return 0;
}

int hakai_deleted(hakai_ctx* c, int64_t* n_deleted, int64_t* log, int64_t cap) {
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    if (!c->model_ok) return fail(HAKAI_ERR_STATE, "deleted before upload_model");
    HIPCHK(hipSetDevice(c->device));
    std::vector<int> ds((size_t)c->nE);
    if (c->nE) HIPCHK(hipMemcpyAsync(ds.data(), c->d_del_step, c->nE * sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    // (step, element) in the reference's print order: by step, then element (v2/HAKAI_j.jl:701-736)
    std::vector<std::pair<long long, long long>> v;
    for (long long e = 0; e < c->nE; ++e)
        if (ds[e] > 0) v.push_back(std::make_pair((long long)ds[e], e + 1 + c->elem_offset));
    std::sort(v.begin(), v.end());
    if (n_deleted) *n_deleted = (int64_t)v.size();
    if (log)
        for (long long i = 0; i < (long long)v.size() && i < cap; ++i) {
            log[2 * i] = v[i].first;
            log[2 * i + 1] = v[i].second;
        }
    return 0;
}

int hakai_set_tuning(hakai_ctx* c, const char* key, int64_t value) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c || !key) return fail(HAKAI_ERR_ARG, "set_tuning: null");
    if (!std::strcmp(key, "elem_pipe_blocks")) {
        if (value < 0 || value > 65536) return fail(HAKAI_ERR_ARG, "elem_pipe_blocks out of range");
        c->pipe_blocks = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "elem_gp_nt")) {
        if (value != 0 && value != 1) return fail(HAKAI_ERR_ARG, "elem_gp_nt must be 0 or 1");
        c->gp_nt = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "fuse_bc")) {
        if (value < 0 || value > 2) return fail(HAKAI_ERR_ARG, "fuse_bc must be 0, 1 or 2 (any mesh size)");
        c->fuse_bc = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "elem_pipe_min")) {
        if (value < 0 || value > 1024) return fail(HAKAI_ERR_ARG, "elem_pipe_min out of range");
        c->pipe_min = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "elem_exact")) {
        if (value != 0 && value != 1) return fail(HAKAI_ERR_ARG, "elem_exact must be 0 or 1");
        if (c->elem_exact != (int)value && c->own_for_g0 != -1) {
            // the owner-assembly plan was sized for the other kernel's LDS budget (the reference-order
            // kernel leaves fewer slots): re-planned before the next step (own_use; one context hands
            // the last sums over through own_materialize). A multi-GPU rank whose sums are live cannot
            // re-plan mid-run (its next interface fix reads the rows): it keeps a plan that fits the
            // new kernel, else the switch is refused.
            if (!(c->comm && c->own_valid)) {
                c->own_for_g0 = -1;
            } else if (c->own_built_g > 0 && c->own_slots > hk::own_slot_cap(value != 0, c->own_s, c->nmat)) {
                return fail(HAKAI_ERR_STATE, "elem_exact: the owner-assembly lists of this multi-GPU rank need %d LDS "
                            "slots, more than the %s kernel has; switch between calls after hakai_upload_state / "
                            "hakai_reset_state", c->own_slots, value ? "reference-order" : "fused");
            }
        }
        c->elem_exact = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "group_serial")) {  // timing: hakai_step_group drains each rank's phase
        if (value < 0 || value > 2) return fail(HAKAI_ERR_ARG, "group_serial must be 0, 1 or 2");
        c->group_serial = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "nodal_padded")) {
        if (!value) {
            dfree(c->d_inc8);
            return 0;
        }
        return c->d_inc8 ? 0 : fail(HAKAI_ERR_STATE, "padded incidence table unavailable (>8 incidences)");
    }
    if (!std::strcmp(key, "own_assembly")) {  // owner-computed node sums in the element kernel
        if (value < 0 || value > 2) return fail(HAKAI_ERR_ARG, "own_assembly must be 0, 1 or 2");
        c->own_assembly = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "own_pass_batches")) {  // batches per owner summing pass (0: planned)
        if (value < 0 || value > 2) return fail(HAKAI_ERR_ARG, "own_pass_batches must be 0, 1 or 2");
        if (c->own_pass_batches != (int)value) c->own_for_g0 = -1;  // re-plan at the next step
        c->own_pass_batches = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "own_band_rows")) {  // row-band height of the banded owner schedule (0: planned)
        if (value < 0 || value > 4096) return fail(HAKAI_ERR_ARG, "own_band_rows must be in [0, 4096]");
        if (c->own_band_rows != (int)value) c->own_for_g0 = -1;  // re-plan at the next step
        c->own_band_rows = (int)value;
        return 0;
    }
    if (!std::strcmp(key, "graph")) {
        if (value < 0 || value > 1024 || (value & 1)) return fail(HAKAI_ERR_ARG, "graph must be 0 or an even step count <= 1024");
        c->graph = (int)value;
        return 0;
    }
    if (!std::strncmp(key, "contact_", 8)) {
        HIPCHK(hipSetDevice(c->device));
        return hkc::contact_tuning(c, key, value);
    }
    return fail(HAKAI_ERR_ARG, "unknown tuning key '%s'", key);
}

int hakai_set_element_offset(hakai_ctx* c, int64_t element_offset) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c || element_offset < 0) return fail(HAKAI_ERR_ARG, "set_element_offset: bad args");
    c->elem_offset = element_offset;
    return 0;
}

int hakai_negative_jacobians(hakai_ctx* c, int64_t* n) {
    if (!c || !n) return fail(HAKAI_ERR_ARG, "null");
    if (!c->state_ok) return fail(HAKAI_ERR_STATE, "negative_jacobians without state");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMemsetAsync(c->d_negjac, 0, sizeof(unsigned long long), c->stream));
    HIPCHK(hk::launch_negjac(elem_args(c), c->d_negjac, c->stream));
    unsigned long long v = 0;
    HIPCHK(hipMemcpyAsync(&v, c->d_negjac, sizeof v, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    *n = (int64_t)v;
    return 0;
}

int hakai_node_stress_strain(hakai_ctx* c, double* node_stress, double* node_strain, double* node_eqps,
                             double* node_mises, double* node_triax) {
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    if (!c->state_ok) return fail(HAKAI_ERR_STATE, "node_stress_strain without state");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const size_t nN = (size_t)c->nN;
    double *ns = nullptr, *nn = nullptr, *ne = nullptr, *nm = nullptr, *nt = nullptr;
    HIPCHK(dalloc(&ns, 6 * nN));
    HIPCHK(dalloc(&nn, 6 * nN));
    HIPCHK(dalloc(&ne, nN));
    HIPCHK(dalloc(&nm, nN));
    HIPCHK(dalloc(&nt, nN));
    HIPCHK(hk::launch_node_average(c->d_inc_ptr, c->d_inc_row, c->d_stress, c->d_strain, c->d_eqps, c->d_triax, c->ld,
                                   c->nN, ns, nn, ne, nm, nt, s));
    if (node_stress) HIPCHK(hipMemcpyAsync(node_stress, ns, 6 * nN * sizeof(double), hipMemcpyDeviceToHost, s));
    if (node_strain) HIPCHK(hipMemcpyAsync(node_strain, nn, 6 * nN * sizeof(double), hipMemcpyDeviceToHost, s));
    if (node_eqps) HIPCHK(hipMemcpyAsync(node_eqps, ne, nN * sizeof(double), hipMemcpyDeviceToHost, s));
    if (node_mises) HIPCHK(hipMemcpyAsync(node_mises, nm, nN * sizeof(double), hipMemcpyDeviceToHost, s));
    if (node_triax) HIPCHK(hipMemcpyAsync(node_triax, nt, nN * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    dfree(ns);
    dfree(nn);
    dfree(ne);
    dfree(nm);
    dfree(nt);
    return 0;
}

int hakai_profile_enable(hakai_ctx* c, int on) { return hakai_profile_mask(c, on ? (1u << HAKAI_K_COUNT) - 1 : 0u); }

int hakai_profile_mask(hakai_ctx* c, uint32_t mask) {
    if (c) hkc::graph_invalidate(c);  // captured steps may hold stale buffers or settings
    if (!c) return fail(HAKAI_ERR_ARG, "null");
    if (!mask) prof_harvest(c);
    c->prof = mask != 0;
    c->prof_mask = mask;
    for (int k = 0; k < HAKAI_K_COUNT; ++k) {
        c->k_ms[k] = 0;
        c->k_n[k] = 0;
    }
    return 0;
}

int hakai_profile_read(hakai_ctx* c, int kernel, double* total_ms, int64_t* launches) {
    if (!c || kernel < 0 || kernel >= HAKAI_K_COUNT) return fail(HAKAI_ERR_ARG, "bad profile query");
    (void)hipSetDevice(c->device);
    prof_harvest(c);
    if (total_ms) *total_ms = c->k_ms[kernel];
    if (launches) *launches = c->k_n[kernel];
    return 0;
}

// ---- stateless literal drop-ins -----------------------------------------------------------------
int hakai_stress_hexa(int device, int64_t nNode, int64_t nElement, double* Qe, double* integ_stress,
                      double* integ_strain, double* integ_yield_stress, double* integ_eq_plastic_strain,
                      const double* position, const double* d_disp, const int64_t* elementmat,
                      const int64_t* element_flag, int32_t integ_num, int32_t nMat, const hakai_material_t* mats,
                      const int64_t* element_material, double* elementVolume) {
    if (integ_num != 8) return fail(HAKAI_ERR_ARG, "integ_num must be 8 (v2/HAKAI_j.jl:177)");
    if (!Qe || !integ_stress || !integ_strain || !integ_yield_stress || !integ_eq_plastic_strain || !position ||
        !d_disp || !element_flag)
        return fail(HAKAI_ERR_ARG, "stress_hexa: null array");
    hakai_ctx* c = nullptr;
    int r = hakai_create(&c, device);
    if (r) return r;
    struct Guard {
        hakai_ctx* c;
        ~Guard() { hakai_destroy(c); }
    } guard{c};
    // position = coord + 0 and d_disp = 0 - (-d_disp): the element kernel reproduces both exactly
    std::vector<double> ones(3 * (size_t)nNode, 1.0);
    r = hakai_upload_model(c, nNode, position, nElement, elementmat, element_material, nMat, mats, ones.data());
    if (r) return r;
    std::vector<double> zero(3 * (size_t)nNode, 0.0), mdu(3 * (size_t)nNode);
    for (size_t i = 0; i < mdu.size(); ++i) mdu[i] = -d_disp[i];
    hakai_state_t st;
    std::memset(&st, 0, sizeof st);
    st.disp = zero.data();
    st.disp_pre = mdu.data();
    st.integ_stress = integ_stress;
    st.integ_strain = integ_strain;
    st.integ_yield_stress = integ_yield_stress;
    st.integ_eq_plastic_strain = integ_eq_plastic_strain;
    st.element_flag = const_cast<int64_t*>(element_flag);
    r = hakai_upload_state(c, &st);
    if (r) return r;
    hipStream_t s = c->stream;
    double* d_vol = nullptr;
    HIPCHK(dalloc(&d_vol, (size_t)c->nEp));
    HIPCHK(hipMemsetAsync(c->d_fe, 0, 24 * (size_t)nElement * sizeof(double), s));
    hk::ElemArgs ea = elem_args(c);
    ea.vol = d_vol;
    ea.pipe_blocks = 0;
    HIPCHK(hk::launch_element(ea, false, false, s));
    std::vector<double> fe(24 * (size_t)nElement), vol((size_t)nElement);
    HIPCHK(hipMemcpyAsync(fe.data(), c->d_fe, fe.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(vol.data(), d_vol, vol.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    dfree(d_vol);
    c->steps_done = 1;
    c->last_dt = 1.0;
    hakai_state_t out;
    std::memset(&out, 0, sizeof out);
    out.integ_stress = integ_stress;
    out.integ_strain = integ_strain;
    out.integ_yield_stress = integ_yield_stress;
    out.integ_eq_plastic_strain = integ_eq_plastic_strain;
    r = hakai_download_state(c, &out);
    if (r) return r;
    for (int64_t e = 0; e < nElement; ++e) {
        if (element_flag[e] == 0) continue;
        for (int j = 0; j < 24; ++j) Qe[24 * e + j] += fe[24 * e + j];
        if (elementVolume) elementVolume[e] = vol[e];
    }
    return 0;
}

int hakai_triax_stress(int device, int64_t nGP, const double* integ_stress, double* integ_triax_stress) {
    if (nGP < 0 || (nGP > 0 && (!integ_stress || !integ_triax_stress))) return fail(HAKAI_ERR_ARG, "triax: bad args");
    int cnt = 0;
    if (hipGetDeviceCount(&cnt) != hipSuccess || cnt <= device || device < 0)
        return fail(HAKAI_ERR_DEVICE, "no HIP device %d: no CPU fallback", device);
    HIPCHK(hipSetDevice(device));
    if (nGP == 0) return 0;
    double *st = nullptr, *tx = nullptr;
    HIPCHK(dalloc(&st, 6 * (size_t)nGP));
    HIPCHK(dalloc(&tx, (size_t)nGP));
    HIPCHK(hipMemcpy(st, integ_stress, 6 * nGP * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hk::launch_triax_aos(st, tx, nGP, 0));
    HIPCHK(hipMemcpy(integ_triax_stress, tx, nGP * sizeof(double), hipMemcpyDeviceToHost));
    dfree(st);
    dfree(tx);
    return 0;
}

}  // extern "C"

// accessors used by other translation units of the library
namespace hkc {
long long ctx_nN(hakai_ctx* c) { return c->nN; }
}
