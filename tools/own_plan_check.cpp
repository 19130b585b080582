// own_plan_check.cpp -- CPU replay of the owner-computed assembly plans (test infrastructure; the
// planner is host code, hakai_capi.cpp own_choose / own_plan, so it is checked here without a GPU).
//
// Builds a structured hex mesh (hakai.mesh.hex_bar numbering: element id x-fastest, C3D8 node
// order), or two of them (plate + impactor, C4's shape), optionally with shuffled element ids, runs
// the planner for one configuration and then REPLAYS the plan exactly as k_element_pipe and k_nodal
// execute it: every block walks its schedule positions, stages its super-batch's contributions by
// lane, runs the super-batch's entries (INIT/continue/FIN sums in LDS slots, exported rows), and the
// nodal side forms own_q[n] + rows in own_ridx order. The result must equal, bit for bit, the
// reference's serial assembly Q[n] = ((0 + c_1) + c_2) + ... in ascending element order
// (v2/HAKAI_j.jl:668-675) for random contributions with mixed signs and magnitudes.
//
//   own_plan_check nx ny nz [--plate px py pz] [--G n] [--exact 0|1] [--schedule 0|1|2]
//                  [--shuffle seed] [--band-rows R]
// Prints one JSON line: {"ok": ..., "planned": ..., "epb", "grid", "superbatch", "banded", "rows",
// "entries", "slots", "mismatch"} and exits 0 when the replay matches (or no plan fits: planned false).
#include "../hakai-fem_amd/csrc/hakai_capi.cpp"

#include <random>

namespace {

void hex_bar(int nx, int ny, int nz, int node0, std::vector<int>& conn) {
    auto id = [&](int x, int y, int z) { return node0 + x + (nx + 1) * (y + (ny + 1) * z); };
    for (int z = 0; z < nz; ++z)
        for (int y = 0; y < ny; ++y)
            for (int x = 0; x < nx; ++x) {
                const int v[8] = {id(x, y, z),         id(x + 1, y, z),         id(x + 1, y + 1, z),
                                  id(x, y + 1, z),     id(x, y, z + 1),         id(x + 1, y, z + 1),
                                  id(x + 1, y + 1, z + 1), id(x, y + 1, z + 1)};
                conn.insert(conn.end(), v, v + 8);
            }
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s nx ny nz [--plate px py pz] [--G n] [--exact e] [--schedule s] "
                     "[--shuffle seed]\n", argv[0]);
        return 2;
    }
    const int nx = std::atoi(argv[1]), ny = std::atoi(argv[2]), nz = std::atoi(argv[3]);
    int px = 0, py = 0, pz = 0, exact = 0, schedule = 0, band_rows = 0;
    long long G0 = 512;
    long long shuffle = -1;
    for (int a = 4; a < argc; ++a) {
        const std::string k = argv[a];
        if (k == "--plate" && a + 3 < argc) {
            px = std::atoi(argv[++a]);
            py = std::atoi(argv[++a]);
            pz = std::atoi(argv[++a]);
        } else if (k == "--G" && a + 1 < argc) G0 = std::atoll(argv[++a]);
        else if (k == "--exact" && a + 1 < argc) exact = std::atoi(argv[++a]);
        else if (k == "--schedule" && a + 1 < argc) schedule = std::atoi(argv[++a]);
        else if (k == "--shuffle" && a + 1 < argc) shuffle = std::atoll(argv[++a]);
        else if (k == "--band-rows" && a + 1 < argc) band_rows = std::atoi(argv[++a]);
        else {
            std::fprintf(stderr, "bad argument %s\n", argv[a]);
            return 2;
        }
    }
    // mesh: [plate] then the bar (two instances, like hakai.mesh.two_body_model)
    std::vector<int> conn;
    int nN = 0;
    if (px > 0) {
        hex_bar(px, py, pz, 0, conn);
        nN = (px + 1) * (py + 1) * (pz + 1);
    }
    hex_bar(nx, ny, nz, nN, conn);
    nN += (nx + 1) * (ny + 1) * (nz + 1);
    long long nE = (long long)conn.size() / 8;
    if (shuffle >= 0) {  // random element numbering
        std::vector<int> perm(nE);
        for (long long e = 0; e < nE; ++e) perm[e] = (int)e;
        std::mt19937_64 rng((unsigned long long)shuffle);
        std::shuffle(perm.begin(), perm.end(), rng);
        std::vector<int> c2(conn.size());
        for (long long e = 0; e < nE; ++e)
            for (int k = 0; k < 8; ++k) c2[8 * e + k] = conn[8 * (size_t)perm[e] + k];
        conn.swap(c2);
    }
    hakai_ctx c;
    c.nE = nE;
    c.nN = nN;
    c.nEp = (nE + 31) / 32 * 32;
    c.h_conn = conn;
    c.nmat = 1;
    c.elem_exact = exact;
    c.own_band_rows = band_rows;
    // node -> (8e + k) CSR in ascending element order (hakai_upload_model)
    std::vector<int> cnt(nN + 1, 0);
    for (long long e = 0; e < nE; ++e)
        for (int k = 0; k < 8; ++k) ++cnt[conn[8 * e + k] + 1];
    int maxinc = 0;
    for (int n = 0; n < nN; ++n) maxinc = std::max(maxinc, cnt[n + 1]);
    for (int n = 0; n < nN; ++n) cnt[n + 1] += cnt[n];
    c.h_ptr = cnt;
    c.h_inc0.assign(8 * (size_t)nE, 0);
    std::vector<int> fill(cnt.begin(), cnt.end() - 1);
    for (long long e = 0; e < nE; ++e)
        for (int k = 0; k < 8; ++k) c.h_inc0[fill[conn[8 * e + k]]++] = (int)(8 * e + k);
    c.max_inc = maxinc;
    const long long G = std::min<long long>(G0, c.nEp / 32);

    OwnSched sc;
    OwnPlan pl;
    const bool planned = own_choose(&c, G, sc, pl, schedule);
    if (!planned) {
        std::printf("{\"ok\": true, \"planned\": false, \"elements\": %lld, \"nodes\": %d}\n", nE, nN);
        return 0;
    }
    // ---- replay (one force component is enough: the three are summed alike)
    const int epb = sc.epb, S = pl.S;
    const long long Gp = (long long)sc.bstart.size() - 1;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> mag(-30.0, 30.0);
    std::vector<double> f(8 * (size_t)c.nEp, 0.0);
    for (long long e = 0; e < nE; ++e)
        for (int k = 0; k < 8; ++k) {
            const double m = std::ldexp(1.0, (int)mag(rng));
            f[8 * e + k] = (rng() & 1 ? -1.0 : 1.0) * m * (1.0 + (double)(rng() >> 11) * 0x1p-53);
        }
    std::vector<double> own_q(nN, 0.0), rows(std::max<long long>(pl.rows, 1), 0.0);
    std::vector<char> q_set(nN, 0);
    std::vector<double> slots(4096, 0.0);
    std::vector<double> stage(8 * (size_t)epb * S);
    auto lane_of = [](const int* w, int j) {
        const unsigned long long lo = (unsigned long long)(unsigned)w[2] | ((unsigned long long)(unsigned)w[3] << 32);
        return j < 7 ? (int)((lo >> (9 * j)) & 511) : (int)(((unsigned)w[1] >> 18) & 511);
    };
    long long bad = 0;
    for (long long lb = 0; lb < Gp; ++lb) {
        for (long long p0 = sc.bstart[lb]; p0 < sc.bstart[lb + 1]; p0 += S) {
            const long long p1 = std::min<long long>(p0 + S, sc.bstart[lb + 1]);
            std::fill(stage.begin(), stage.end(), 0.0);
            for (long long p = p0; p < p1; ++p)
                for (int l = 0; l < 8 * epb; ++l) {
                    const long long e = (long long)sc.seq[p] * epb + l / 8;
                    stage[(p - p0) * 8 * epb + l] = e < nE ? f[8 * e + l % 8] : 0.0;
                }
            for (int q = pl.off[p0]; q < pl.off[p0 + 1]; ++q) {
                const int* w = &pl.list[4 * (size_t)q];
                const int slot = (w[1] & 1023) | ((w[1] >> 18) & 1024), flags = (w[1] >> 10) & 15,
                          n = (w[1] >> 14) & 15;
                if (flags & kOwnExpH) {
                    for (int j = 0; j < n; ++j) rows[w[0] + (long long)j * slot] = stage[lane_of(w, j)];
                    continue;
                }
                if (flags & kOwnNopH) continue;
                double v = (flags & kOwnInitH) ? 0.0 : slots[slot];
                for (int j = 0; j < n; ++j) v += stage[lane_of(w, j)];
                if (flags & kOwnFinH) {
                    if (q_set[w[0]]) ++bad;  // a node's sum is finished once
                    q_set[w[0]] = 1;
                    own_q[w[0]] = v;
                } else {
                    slots[slot] = v;
                }
            }
        }
    }
    long long mismatch = 0;
    for (int n = 0; n < nN; ++n) {
        double ref = 0.0;
        for (int j = c.h_ptr[n]; j < c.h_ptr[n + 1]; ++j) ref += f[c.h_inc0[j]];
        double q = own_q[n];
        for (int r = pl.rp[n]; r < pl.rp[n + 1]; ++r) q += rows[pl.ridx[r]];
        if (std::memcmp(&q, &ref, sizeof q) != 0) ++mismatch;
    }
    const bool ok = mismatch == 0 && bad == 0;
    std::printf("{\"ok\": %s, \"planned\": true, \"elements\": %lld, \"nodes\": %d, \"epb\": %d, \"grid\": %lld, "
                "\"superbatch\": %d, \"banded\": %d, \"rows\": %lld, \"entries\": %lld, \"slots\": %d, "
                "\"slot_cap\": %d, \"round2\": %lld, \"mismatch\": %lld, \"double_fin\": %lld}\n",
                ok ? "true" : "false", nE, nN, epb, Gp, S, sc.banded ? 1 : 0, pl.rows, pl.ne, pl.max_slots,
                hk::own_slot_cap(exact != 0, S, 1), pl.round2, mismatch, bad);
    return ok ? 0 : 1;
}
