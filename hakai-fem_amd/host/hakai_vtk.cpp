// hakai_vtk.cpp -- the legacy-ASCII VTK output of HAKAI (write_vtk, v2/HAKAI_j.jl:3517-3717), written
// in parallel and off the time loop's critical path.
//
// The reference formats every value with @printf "%1.6e" on one thread and the time loop waits for
// it (v2/HAKAI_j.jl:932-942). At C3 size (2.2 M nodes, 23 values per node) one file is ~0.7 GB of
// text, so a synchronous serial writer costs seconds per output, 100 outputs per run, while the
// device needs about a millisecond per step. Here:
//   * numbers are formatted with std::to_chars(scientific, 6), which the C++ standard defines as
//     printf's "%.6e" in the C locale (byte-identical, checked against snprintf in
//     tests/test_vtk.py), ~3.5x faster than snprintf per value;
//   * a file is cut into node / element ranges formatted by a team of threads, then written in
//     order with large fwrites;
//   * the constant POINTS block (initial coordinates, :3574-3577) is formatted once per writer;
//   * hakai_vtk_writer_submit() (or acquire/commit, zero-copy) snapshots the arrays and returns;
//     the file is written by a background thread while the caller keeps stepping the device.
// The file content is exactly the serial writer's: same sections, same order, same tiny-value
// flush (|x| < 1e-16 -> 0, :3530-3558), cells of live elements only, 0-based node ids.
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <sys/stat.h>
#include <thread>
#include <vector>

#include "../../include/hakai_hip.h"

namespace hkc {
int fail(int code, const char* fmt, ...);
}
using hkc::fail;

namespace {

inline double flush16(double x) { return std::fabs(x) < 1E-16 ? 0.0 : x; }

// "%1.6e": at most "-1.234567e-308" = 14 chars
constexpr int kMaxNum = 16;

// Julia's @printf prints non-finite values as "NaN", "Inf" and "-Inf" (C's printf: "nan", "inf")
inline char* put_e(char* p, double x) {
    if (!std::isfinite(x)) {
        const char* t = std::isnan(x) ? "NaN" : (x > 0 ? "Inf" : "-Inf");
        while (*t) *p++ = *t++;
        return p;
    }
    return std::to_chars(p, p + kMaxNum, x, std::chars_format::scientific, 6).ptr;
}

inline char* put_i(char* p, long long v) { return std::to_chars(p, p + 24, v).ptr; }

int default_threads() {
    const char* e = std::getenv("HAKAI_VTK_THREADS");
    if (!e || !*e) e = std::getenv("OMP_NUM_THREADS");
    int n = e && *e ? std::atoi(e) : 0;
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(n, 64));
}

template <class F>
void parallel_ranges(int nt, int64_t n, F&& f) {
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, (n + 4095) / 4096));
    if (nt == 1) {
        f(0, (int64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(nt - 1);
    for (int t = 1; t < nt; ++t) th.emplace_back([&, t] { f(t, n * t / nt, n * (t + 1) / nt); });
    f(0, (int64_t)0, n / nt);
    for (auto& x : th) x.join();
}

struct Buf {  // one thread's text for one section
    std::vector<char> b;
    size_t n = 0;
    char* reserve(size_t cap) {
        if (b.size() < cap) b.resize(cap);
        n = 0;
        return b.data();
    }
};

// The per-output arrays (disp, velo: 3 x nN; node stress/strain: 6 x nN; the rest nN).
struct Snapshot {
    std::vector<int64_t> flag;
    std::vector<double> disp, velo, ns, nn, ne, nm, nt;
};

}  // namespace

struct hakai_vtk_writer {
    int threads = 1;
    std::string dir;
    int64_t nN = 0, nE = 0;
    std::vector<int64_t> elementmat;  // 8 x nE, 1-based (copied)
    std::string points;               // "POINTS ...\n" + coordinates, formatted once
    // per-thread section buffers, reused across files: [section][thread]
    std::vector<std::vector<Buf>> sec;
    std::vector<Buf> cells;
    std::vector<long long> draw_part;
    Snapshot snap;  // being written by `worker`
    Snapshot fill;  // being filled by the caller (acquire/commit)
    std::thread worker;
    bool busy = false;
    int status = 0;
    std::string err;

    int write_file(int index);
};

namespace {

// Section table after POINT_DATA (v2/HAKAI_j.jl:3597-3712): name, source array, stride, component.
struct SecDef {
    const char* head;  // full header text
    int src;           // 0 disp(vec3) 1 velo 2 strain 3 eqps 4 stress 5 mises 6 triax
    int comp;
};
const SecDef kSecs[] = {
    {"VECTORS DISPLACEMENT float\n", 0, -1},
    {"SCALARS Vx float 1\nLOOKUP_TABLE default\n", 1, 0},
    {"SCALARS Vy float 1\nLOOKUP_TABLE default\n", 1, 1},
    {"SCALARS Vz float 1\nLOOKUP_TABLE default\n", 1, 2},
    {"SCALARS E11 float 1\nLOOKUP_TABLE default\n", 2, 0},
    {"SCALARS E22 float 1\nLOOKUP_TABLE default\n", 2, 1},
    {"SCALARS E33 float 1\nLOOKUP_TABLE default\n", 2, 2},
    {"SCALARS E12 float 1\nLOOKUP_TABLE default\n", 2, 3},
    {"SCALARS E23 float 1\nLOOKUP_TABLE default\n", 2, 4},
    {"SCALARS E13 float 1\nLOOKUP_TABLE default\n", 2, 5},
    {"SCALARS EQ_PSTRAIN float 1\nLOOKUP_TABLE default\n", 3, 0},
    {"SCALARS S11 float 1\nLOOKUP_TABLE default\n", 4, 0},
    {"SCALARS S22 float 1\nLOOKUP_TABLE default\n", 4, 1},
    {"SCALARS S33 float 1\nLOOKUP_TABLE default\n", 4, 2},
    {"SCALARS S12 float 1\nLOOKUP_TABLE default\n", 4, 3},
    {"SCALARS S23 float 1\nLOOKUP_TABLE default\n", 4, 4},
    {"SCALARS S13 float 1\nLOOKUP_TABLE default\n", 4, 5},
    {"SCALARS MISES_STRESS float 1\nLOOKUP_TABLE default\n", 5, 0},
    {"SCALARS TRIAX_STRESS float 1\nLOOKUP_TABLE default\n", 6, 0},
};
constexpr int kNSec = sizeof(kSecs) / sizeof(kSecs[0]);

bool put_all(FILE* f, const char* p, size_t n) { return n == 0 || std::fwrite(p, 1, n, f) == n; }

}  // namespace

int hakai_vtk_writer::write_file(int index) {
    const Snapshot& s = snap;
    const int T = threads;
    sec.resize(kNSec);
    for (auto& v : sec) v.resize(T);
    cells.resize(T);
    draw_part.assign(T, 0);
    for (auto& v : sec)
        for (auto& b : v) b.n = 0;  // ranges a small mesh leaves unused stay empty
    for (auto& b : cells) b.n = 0;
    // cells of live elements (:3579-3588), element ranges per thread
    parallel_ranges(T, nE, [&](int t, int64_t lo, int64_t hi) {
        char* p0 = cells[t].reserve((size_t)(hi - lo) * (2 + 8 * 21) + 1);
        char* p = p0;
        long long d = 0;
        for (int64_t e = lo; e < hi; ++e) {
            d += s.flag[e];
            if (s.flag[e] != 1) continue;
            const int64_t* c = elementmat.data() + 8 * e;
            *p++ = '8';
            for (int i = 0; i < 8; ++i) {
                *p++ = ' ';
                p = put_i(p, (long long)c[i] - 1);
            }
            *p++ = '\n';
        }
        cells[t].n = (size_t)(p - p0);
        draw_part[t] = d;
    });
    // node sections, node ranges per thread
    parallel_ranges(T, nN, [&](int t, int64_t lo, int64_t hi) {
        const size_t cnt = (size_t)(hi - lo);
        for (int k = 0; k < kNSec; ++k) {
            const SecDef& d = kSecs[k];
            Buf& B = sec[k][t];
            char* p0 = B.reserve(cnt * (d.src == 0 ? 3 * (kMaxNum + 1) : kMaxNum + 1));
            char* p = p0;
            switch (d.src) {
                case 0:
                    for (int64_t i = lo; i < hi; ++i) {
                        p = put_e(p, flush16(s.disp[3 * i]));
                        *p++ = ' ';
                        p = put_e(p, flush16(s.disp[3 * i + 1]));
                        *p++ = ' ';
                        p = put_e(p, flush16(s.disp[3 * i + 2]));
                        *p++ = '\n';
                    }
                    break;
                case 1:
                    for (int64_t i = lo; i < hi; ++i) p = put_e(p, flush16(s.velo[3 * i + d.comp])), *p++ = '\n';
                    break;
                case 2:
                    for (int64_t i = lo; i < hi; ++i) p = put_e(p, flush16(s.nn[6 * i + d.comp])), *p++ = '\n';
                    break;
                case 3:
                    for (int64_t i = lo; i < hi; ++i) p = put_e(p, flush16(s.ne[i])), *p++ = '\n';
                    break;
                case 4:
                    for (int64_t i = lo; i < hi; ++i) p = put_e(p, flush16(s.ns[6 * i + d.comp])), *p++ = '\n';
                    break;
                case 5:
                    for (int64_t i = lo; i < hi; ++i) p = put_e(p, flush16(s.nm[i])), *p++ = '\n';
                    break;
                default:
                    for (int64_t i = lo; i < hi; ++i) p = put_e(p, flush16(s.nt[i])), *p++ = '\n';
                    break;
            }
            B.n = (size_t)(p - p0);
        }
    });
    long long draw = 0;
    for (long long d : draw_part) draw += d;

    mkdir(dir.c_str(), 0755);
    char fname[4096];
    std::snprintf(fname, sizeof fname, "%s/file%03d.vtk", dir.c_str(), index);
    FILE* f = std::fopen(fname, "w");
    if (!f) {
        err = std::string("cannot write ") + fname;
        return HAKAI_ERR_IO;
    }
    std::setvbuf(f, nullptr, _IONBF, 0);  // our buffers are large already
    bool ok = true;
    char hdr[256];
    ok = ok && put_all(f, points.data(), points.size());
    int h = std::snprintf(hdr, sizeof hdr, "CELLS %lld %lld\n", draw, draw * (8 + 1));
    ok = ok && put_all(f, hdr, (size_t)h);
    for (auto& b : cells) ok = ok && put_all(f, b.b.data(), b.n);
    h = std::snprintf(hdr, sizeof hdr, "CELL_TYPES %lld\n", draw);
    ok = ok && put_all(f, hdr, (size_t)h);
    {
        std::string types;
        const long long chunk = 1 << 20;
        for (long long i = 0; i < draw; i += chunk) {
            const long long m = std::min(chunk, draw - i);
            types.resize(3 * (size_t)m);
            for (long long j = 0; j < m; ++j) std::memcpy(&types[3 * j], "12\n", 3);
            ok = ok && put_all(f, types.data(), types.size());
        }
    }
    h = std::snprintf(hdr, sizeof hdr, "POINT_DATA %lld\n", (long long)nN);
    ok = ok && put_all(f, hdr, (size_t)h);
    for (int k = 0; k < kNSec; ++k) {
        ok = ok && put_all(f, kSecs[k].head, std::strlen(kSecs[k].head));
        for (auto& b : sec[k]) ok = ok && put_all(f, b.b.data(), b.n);
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok) {
        err = std::string("write failed: ") + fname;
        return HAKAI_ERR_IO;
    }
    return 0;
}

namespace {

int check_arrays(const int64_t* flag, const double* disp, const double* velo, const double* ns, const double* nn,
                 const double* ne, const double* nm, const double* nt) {
    if (!flag || !disp || !velo || !ns || !nn || !ne || !nm || !nt) return fail(HAKAI_ERR_ARG, "write_vtk: null array");
    return 0;
}

void size_snapshot(Snapshot& s, int64_t nN, int64_t nE) {
    const size_t N = (size_t)nN;
    s.flag.resize((size_t)nE);
    s.disp.resize(3 * N);
    s.velo.resize(3 * N);
    s.ns.resize(6 * N);
    s.nn.resize(6 * N);
    s.ne.resize(N);
    s.nm.resize(N);
    s.nt.resize(N);
}

void copy_into(Snapshot& s, int64_t nN, int64_t nE, const int64_t* flag, const double* disp, const double* velo,
               const double* ns, const double* nn, const double* ne, const double* nm, const double* nt) {
    const size_t N = (size_t)nN;
    s.flag.assign(flag, flag + nE);
    s.disp.assign(disp, disp + 3 * N);
    s.velo.assign(velo, velo + 3 * N);
    s.ns.assign(ns, ns + 6 * N);
    s.nn.assign(nn, nn + 6 * N);
    s.ne.assign(ne, ne + N);
    s.nm.assign(nm, nm + N);
    s.nt.assign(nt, nt + N);
}

}  // namespace

extern "C" {

int hakai_vtk_writer_create(hakai_vtk_writer** out, const char* dir, int64_t nNode, const double* coordmat,
                            int64_t nElement, const int64_t* elementmat, int n_threads) {
    if (!out || !dir || nNode < 0 || nElement < 0 || (nNode > 0 && !coordmat) || (nElement > 0 && !elementmat))
        return fail(HAKAI_ERR_ARG, "vtk_writer_create: bad arguments");
    *out = nullptr;
    hakai_vtk_writer* w = new hakai_vtk_writer();
    w->threads = n_threads > 0 ? std::min(n_threads, 64) : default_threads();
    w->dir = dir;
    w->nN = nNode;
    w->nE = nElement;
    w->elementmat.assign(elementmat, elementmat + 8 * nElement);
    // header + POINTS (:3566-3577): initial coordinates, constant over the run
    std::string& P = w->points;
    char hdr[256];
    const int h = std::snprintf(hdr, sizeof hdr,
                                "# vtk DataFile Version 2.0\nTest\nASCII\nDATASET UNSTRUCTURED_GRID\nPOINTS %lld float\n",
                                (long long)nNode);
    std::vector<Buf> pb(w->threads);
    parallel_ranges(w->threads, nNode, [&](int t, int64_t lo, int64_t hi) {
        char* p0 = pb[t].reserve((size_t)(hi - lo) * 3 * (kMaxNum + 1));
        char* p = p0;
        for (int64_t i = lo; i < hi; ++i) {
            p = put_e(p, coordmat[3 * i]);
            *p++ = ' ';
            p = put_e(p, coordmat[3 * i + 1]);
            *p++ = ' ';
            p = put_e(p, coordmat[3 * i + 2]);
            *p++ = '\n';
        }
        pb[t].n = (size_t)(p - p0);
    });
    size_t tot = (size_t)h;
    for (auto& b : pb) tot += b.n;
    P.reserve(tot);
    P.append(hdr, (size_t)h);
    for (auto& b : pb) P.append(b.b.data(), b.n);
    *out = w;
    return 0;
}

int hakai_vtk_writer_wait(hakai_vtk_writer* w) {
    if (!w) return fail(HAKAI_ERR_ARG, "vtk_writer_wait: null writer");
    if (w->busy) {
        w->worker.join();
        w->busy = false;
    }
    if (w->status) {
        const int st = w->status;
        w->status = 0;
        return fail(st, "write_vtk: %s", w->err.c_str());
    }
    return 0;
}

int hakai_vtk_writer_acquire(hakai_vtk_writer* w, hakai_vtk_arrays_t* a) {
    if (!w || !a) return fail(HAKAI_ERR_ARG, "vtk_writer_acquire: null argument");
    size_snapshot(w->fill, w->nN, w->nE);
    Snapshot& s = w->fill;
    a->element_flag = s.flag.data();
    a->disp = s.disp.data();
    a->velo = s.velo.data();
    a->node_stress = s.ns.data();
    a->node_strain = s.nn.data();
    a->node_eq_plastic_strain = s.ne.data();
    a->node_mises_stress = s.nm.data();
    a->node_triax_stress = s.nt.data();
    return 0;
}

int hakai_vtk_writer_commit(hakai_vtk_writer* w, int index) {
    if (!w) return fail(HAKAI_ERR_ARG, "vtk_writer_commit: null writer");
    int r = hakai_vtk_writer_wait(w);  // the previous file's error surfaces here
    if (r) return r;
    std::swap(w->snap, w->fill);
    w->busy = true;
    w->worker = std::thread([w, index] { w->status = w->write_file(index); });
    return 0;
}

int hakai_vtk_writer_submit(hakai_vtk_writer* w, int index, const int64_t* element_flag, const double* disp,
                            const double* velo, const double* node_stress, const double* node_strain,
                            const double* node_eq_plastic_strain, const double* node_mises_stress,
                            const double* node_triax_stress) {
    if (!w) return fail(HAKAI_ERR_ARG, "vtk_writer_submit: null writer");
    int r = check_arrays(element_flag, disp, velo, node_stress, node_strain, node_eq_plastic_strain,
                         node_mises_stress, node_triax_stress);
    if (r) return r;
    copy_into(w->fill, w->nN, w->nE, element_flag, disp, velo, node_stress, node_strain, node_eq_plastic_strain,
              node_mises_stress, node_triax_stress);
    return hakai_vtk_writer_commit(w, index);
}

void hakai_vtk_writer_destroy(hakai_vtk_writer* w) {
    if (!w) return;
    if (w->busy) w->worker.join();
    delete w;
}

int hakai_write_vtk(const char* dir, int index, int64_t nNode, const double* coordmat, int64_t nElement,
                    const int64_t* elementmat, const int64_t* element_flag, const double* disp, const double* velo,
                    const double* node_stress, const double* node_strain, const double* node_eqps,
                    const double* node_mises, const double* node_triax) {
    if (!dir || !coordmat || !elementmat) return fail(HAKAI_ERR_ARG, "write_vtk: null array");
    int r = check_arrays(element_flag, disp, velo, node_stress, node_strain, node_eqps, node_mises, node_triax);
    if (r) return r;
    hakai_vtk_writer* w = nullptr;
    if ((r = hakai_vtk_writer_create(&w, dir, nNode, coordmat, nElement, elementmat, 0))) return r;
    copy_into(w->snap, nNode, nElement, element_flag, disp, velo, node_stress, node_strain, node_eqps, node_mises,
              node_triax);
    r = w->write_file(index);
    if (r) r = fail(r, "write_vtk: %s", w->err.c_str());
    hakai_vtk_writer_destroy(w);
    return r;
}

}  // extern "C"
