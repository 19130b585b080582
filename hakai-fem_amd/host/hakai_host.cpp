// hakai_host.cpp -- driver surface of HAKAI on MI355X: the Abaqus-subset .inp reader
// (readInpFile, v2/readInpFile_j.jl:152-1113), model setup (lumped mass, v2/HAKAI_j.jl:183-218),
// the legacy VTK writer (write_vtk, v2/HAKAI_j.jl:3517-3717) and HAKAI(fname) itself
// (v2/HAKAI_j.jl:81-978), which drives the device time loop through the C ABI.
//
// The reader reproduces the reference's line-matching semantics, including its quirks
// (SURVEY.md §9): a multi-line *Amplitude keeps only its last line; assembly *Nset lookups for
// *Boundary append every match while *Initial Conditions take the first; ENCASTRE fixes the 3 dofs;
// directions > 3 are ignored; a BC block ends at "**" or the next "*Boundary".
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "../../include/hakai_hip.h"

namespace hkc {
int fail(int code, const char* fmt, ...);
}
using hkc::fail;

namespace {

struct ParseError {
    std::string msg;
};

std::string nospace(const std::string& s) {  // replace(s, " " => "")
    std::string o;
    o.reserve(s.size());
    for (char ch : s)
        if (ch != ' ') o.push_back(ch);
    return o;
}

// split(s, ",", keepempty=false) / keepempty=true
std::vector<std::string> split(const std::string& s, char d, bool keepempty) {
    std::vector<std::string> out;
    std::string cur;
    for (char ch : s) {
        if (ch == d) {
            if (keepempty || !cur.empty()) out.push_back(cur);
            cur.clear();
        } else {
            cur.push_back(ch);
        }
    }
    if (keepempty || !cur.empty()) out.push_back(cur);
    return out;
}

bool has(const std::string& s, const char* pat) { return s.find(pat) != std::string::npos; }

// Julia's parse(Float64 / Int, s) accepts leading and trailing whitespace (tabs in decks written
// by spreadsheets, e.g. HAKAI-v0.0.1/input/projectile-impact-d1mm.inp *Plastic rows)
static std::string trim_ws(const std::string& s) {
    size_t a = 0, b = s.size();
    while (a < b && std::isspace((unsigned char)s[a])) ++a;
    while (b > a && std::isspace((unsigned char)s[b - 1])) --b;
    return s.substr(a, b - a);
}

double parse_f(const std::string& s0) {
    const std::string s = trim_ws(s0);
    if (s.empty()) throw ParseError{"parse(Float64, \"" + s0 + "\")"};
    char* end = nullptr;
    const double v = std::strtod(s.c_str(), &end);
    if (end != s.c_str() + s.size()) throw ParseError{"parse(Float64, \"" + s0 + "\")"};
    return v;
}

long long parse_i(const std::string& s0) {
    const std::string s = trim_ws(s0);
    if (s.empty()) throw ParseError{"parse(Int, \"" + s0 + "\")"};
    char* end = nullptr;
    const long long v = std::strtoll(s.c_str(), &end, 10);
    if (end != s.c_str() + s.size()) throw ParseError{"parse(Int, \"" + s0 + "\")"};
    return v;
}

std::string after(const std::string& s, const char* key) {  // ss[findfirst(key, ss).stop+1 : end]
    const size_t p = s.find(key);
    if (p == std::string::npos) throw ParseError{std::string("keyword '") + key + "' not found in '" + s + "'"};
    return s.substr(p + std::strlen(key));
}

const std::string& at(const std::vector<std::string>& v, size_t i1) {  // 1-based with bounds error
    if (i1 < 1 || i1 > v.size()) throw ParseError{"BoundsError on token list"};
    return v[i1 - 1];
}

std::vector<long long> range_line(const std::vector<std::string>& ss) {  // a:c:b
    const long long a = parse_i(at(ss, 1)), b = parse_i(at(ss, 2)), c = parse_i(at(ss, 3));
    std::vector<long long> r;
    if (c == 0) throw ParseError{"zero step range"};
    if (c > 0)
        for (long long j = a; j <= b; j += c) r.push_back(j);
    else
        for (long long j = a; j >= b; j += c) r.push_back(j);
    return r;
}

struct Nset {
    std::string name, instance_name, part_name;
    int instance_id = 0, part_id = 0;  // 1-based, 0 = none
    std::vector<long long> nodes;
};
struct Part {
    std::string name;
    long long nNode = 0, nElement = 0;
    std::vector<double> coord;     // 3 x nNode
    std::vector<long long> elem;   // 8 x nElement
    std::vector<Nset> nsets;
    std::string material_name;
    int material_id = 0;
};
struct Instance {
    std::string name, part_name;
    int part_id = 0, material_id = 0;
    std::vector<std::string> translate;
    long long node_offset = 0, nNode = 0, element_offset = 0, nElement = 0;
};
struct Elset {
    std::string name, instance_name, part_name;
    int instance_id = 0, part_id = 0;
    std::vector<long long> elements;
};
struct Amp {
    std::string name;
    std::vector<double> time{0.0}, value{0.0};
};
struct Mat {
    std::string name;
    double density = 0, young = 0, poisson = 0, failure_stress = 0;
    int fracture_flag = 0;
    std::vector<double> plastic;  // [n][2]
    std::vector<double> ductile;  // [n][3]
};
struct BC {
    std::string amp_name;
    Amp amp;
    std::vector<std::vector<long long>> dof;
    std::vector<double> value;
};
struct IC {
    std::vector<std::vector<long long>> dof;
    std::vector<double> value;
};

struct Owned {
    hakai_inp_model_t pub;
    std::vector<double> coord;
    std::vector<int64_t> elem, emat, einst;
    std::vector<hakai_material_t> mats;
    std::vector<std::vector<double>> mat_pl, mat_du;
    std::vector<int32_t> amp_n;
    std::vector<int64_t> amp_off, entry_off, dof_off, dofs, ic_dofs;
    std::vector<double> amp_t, amp_v, entry_val, ic_val;
    std::vector<int64_t> inst_noff, inst_eoff, inst_ne;
    std::vector<int32_t> cp_inst;           // *Contact Pair: 2 instances per pair
    std::vector<int64_t> cp_off, cp_elems;  // surface element lists (instance-local, 1-based)
};

void read_lines(const char* path, std::vector<std::string>& lines) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw ParseError{std::string("cannot open ") + path};
    std::string l;
    while (std::getline(f, l)) {
        if (!l.empty() && l.back() == '\r') l.pop_back();
        lines.push_back(l);
    }
}

void parse(const char* path, Owned& o) {
    std::vector<std::string> L;
    read_lines(path, L);
    const long long n = (long long)L.size();
    auto line = [&](long long i1) -> const std::string& {  // 1-based
        if (i1 < 1 || i1 > n) throw ParseError{"BoundsError: line index past end of file"};
        return L[i1 - 1];
    };

    // ---- Part (v2/readInpFile_j.jl:165-308)
    std::vector<long long> part_index;
    for (long long i = 1; i <= n; ++i)
        if (has(line(i), "*Part, name=")) part_index.push_back(i);
    std::vector<Part> PART(part_index.size());
    for (size_t k = 0; k < PART.size(); ++k) {
        Part& P = PART[k];
        auto ss = split(nospace(line(part_index[k])), ',', false);
        P.name = after(at(ss, 2), "name=");
        long long index = 1;
        for (long long i = part_index[k]; i <= n; ++i)
            if (has(line(i), "*Node")) {
                index = i;
                break;
            }
        long long nNode = 0;
        for (long long i = index + 1; i <= n; ++i) {
            if (has(line(i), "*")) break;
            ++nNode;
        }
        P.nNode = nNode;
        P.coord.assign(3 * (size_t)nNode, 0.0);
        for (long long i = 1; i <= nNode; ++i) {
            auto t = split(nospace(line(index + i)), ',', false);
            P.coord[3 * (i - 1) + 0] = parse_f(at(t, 2));
            P.coord[3 * (i - 1) + 1] = parse_f(at(t, 3));
            P.coord[3 * (i - 1) + 2] = parse_f(at(t, 4));
        }
        index = 1;
        for (long long i = part_index[k]; i <= n; ++i)
            if (has(line(i), "*Element")) {
                index = i;
                break;
            }
        long long nEl = 0;
        for (long long i = index + 1; i <= n; ++i) {
            if (has(line(i), "*")) break;
            ++nEl;
        }
        P.nElement = nEl;
        P.elem.assign(8 * (size_t)nEl, 0);
        for (long long i = 1; i <= nEl; ++i) {
            auto t = split(nospace(line(index + i)), ',', false);
            for (int j = 1; j <= 8; ++j) P.elem[8 * (i - 1) + (j - 1)] = parse_i(at(t, 1 + j));
        }
        std::vector<long long> nset_index;
        for (long long i = part_index[k]; i <= n; ++i) {
            if (has(line(i), "*Nset") && has(line(i), "generate")) nset_index.push_back(i);
            if (has(line(i), "*End Part")) break;
        }
        for (long long ni : nset_index) {
            Nset ns;
            auto t = split(nospace(line(ni)), ',', false);
            ns.name = after(at(t, 2), "nset=");
            auto r = split(nospace(line(ni + 1)), ',', true);
            ns.nodes = range_line(r);
            P.nsets.push_back(ns);
        }
        for (long long i = part_index[k]; i <= n; ++i) {
            if (has(line(i), "*Solid Section")) {
                auto t = split(nospace(line(i)), ',', false);
                for (auto& s3 : t)
                    if (has(s3, "material=")) {
                        P.material_name = after(s3, "material=");
                        break;
                    }
                break;
            }
        }
    }

    // ---- Instance (:311-362)
    std::vector<long long> instance_index;
    for (long long i = 1; i <= n; ++i)
        if (has(line(i), "*Instance")) instance_index.push_back(i);
    std::vector<Instance> INST(instance_index.size());
    for (size_t k = 0; k < INST.size(); ++k) {
        auto ss = split(nospace(line(instance_index[k])), ',', false);
        INST[k].name = after(at(ss, 2), "name=");
        INST[k].part_name = after(at(ss, 3), "part=");
        for (size_t i = 0; i < PART.size(); ++i)
            if (PART[i].name == INST[k].part_name) {
                INST[k].part_id = (int)i + 1;
                break;
            }
        for (long long i = instance_index[k] + 1; i <= n; ++i) {
            if (has(line(i), "*End Instance")) break;
            INST[k].translate.push_back(nospace(line(i)));
        }
    }

    // ---- assembly Nset (:365-432)
    std::vector<Nset> NSET;
    for (long long i = 1; i <= n; ++i) {
        if (!(has(line(i), "*Nset") && has(line(i), "instance="))) continue;
        Nset ns;
        const std::string s = nospace(line(i));
        auto ss = split(s, ',', false);
        ns.name = after(at(ss, 2), "nset=");
        ns.instance_name = after(at(ss, 3), "instance=");
        for (size_t j = 0; j < INST.size(); ++j)
            if (ns.instance_name == INST[j].name) {
                ns.part_name = INST[j].part_name;
                ns.part_id = INST[j].part_id;
                ns.instance_id = (int)j + 1;
            }
        if (ss.size() == 4 && ss[3] == "generate") {
            ns.nodes = range_line(split(nospace(line(i + 1)), ',', false));
        } else {
            for (long long r = i + 1; r <= n; ++r) {
                if (has(line(r), "*")) break;
                for (auto& tok : split(nospace(line(r)), ',', false)) ns.nodes.push_back(parse_i(tok));
            }
        }
        NSET.push_back(ns);
    }

    // ---- Elset (:435-515)
    std::vector<Elset> ELSET;
    for (long long i = 1; i <= n; ++i) {
        if (!(has(line(i), "*Elset") && has(line(i), "instance="))) continue;
        Elset es;
        const std::string s = nospace(line(i));
        auto ss = split(s, ',', false);
        es.name = after(at(ss, 2), "elset=");
        if (has(at(ss, 3), "instance=")) es.instance_name = after(ss[2], "instance=");
        else if (has(at(ss, 4), "instance=")) es.instance_name = after(ss[3], "instance=");
        for (size_t j = 0; j < INST.size(); ++j)
            if (es.instance_name == INST[j].name) {
                es.part_name = INST[j].part_name;
                es.part_id = INST[j].part_id;
                es.instance_id = (int)j + 1;
            }
        if (ss.size() == 4 && ss[3] == "generate") {
            es.elements = range_line(split(nospace(line(i + 1)), ',', false));
        } else if (ss.size() == 5 && ss[2] == "internal" && ss[4] == "generate") {
            es.elements = range_line(split(nospace(line(i + 1)), ',', false));
        } else if (ss.size() == 4 && ss[2] == "internal") {
            for (long long r = i + 1; r <= n; ++r) {
                if (has(line(r), "*")) break;
                for (auto& tok : split(nospace(line(r)), ',', false)) es.elements.push_back(parse_i(tok));
            }
        }
        ELSET.push_back(es);
    }
    (void)ELSET;  // surfaces / contact pairs: consumed by the contact path

    // ---- global model (:567-621)
    long long nNode = 0, nElement = 0;
    std::vector<double> coordmat;
    std::vector<long long> elementmat;
    for (size_t i = 0; i < INST.size(); ++i) {
        Instance& I = INST[i];
        if (I.part_id == 0) throw ParseError{"instance part not found: " + I.part_name};
        const Part& P = PART[I.part_id - 1];
        std::vector<double> ci = P.coord;
        I.node_offset = nNode;
        I.element_offset = nElement;
        I.nNode = P.nNode;
        I.nElement = P.nElement;
        for (long long j = (long long)I.translate.size(); j >= 1; --j) {
            auto ss = split(I.translate[j - 1], ',', false);
            if (ss.size() == 3) {
                const double ox = parse_f(ss[0]), oy = parse_f(ss[1]), oz = parse_f(ss[2]);
                for (long long q = 0; q < P.nNode; ++q) {
                    ci[3 * q + 0] = ci[3 * q + 0] + ox * 1.0;
                    ci[3 * q + 1] = ci[3 * q + 1] + oy * 1.0;
                    ci[3 * q + 2] = ci[3 * q + 2] + oz * 1.0;
                }
            } else if (ss.size() == 7) {
                double nv[3] = {parse_f(ss[3]) - parse_f(ss[0]), parse_f(ss[4]) - parse_f(ss[1]),
                                parse_f(ss[5]) - parse_f(ss[2])};
                const double nrm = std::sqrt(nv[0] * nv[0] + nv[1] * nv[1] + nv[2] * nv[2]);
                for (double& x : nv) x = x / nrm;
                const double n1 = nv[0], n2 = nv[1], n3 = nv[2];
                const double d = parse_f(ss[6]) / 180.0 * M_PI;
                const double T[3][3] = {
                    {n1 * n1 * (1 - std::cos(d)) + std::cos(d), n1 * n2 * (1 - std::cos(d)) - n3 * std::sin(d),
                     n1 * n3 * (1 - std::cos(d)) + n2 * std::sin(d)},
                    {n1 * n2 * (1 - std::cos(d)) + n3 * std::sin(d), n2 * n2 * (1 - std::cos(d)) + std::cos(d),
                     n2 * n3 * (1 - std::cos(d)) - n1 * std::sin(d)},
                    {n1 * n3 * (1 - std::cos(d)) - n2 * std::sin(d), n2 * n3 * (1 - std::cos(d)) + n1 * std::sin(d),
                     n3 * n3 * (1 - std::cos(d)) + std::cos(d)}};
                for (long long q = 0; q < P.nNode; ++q) {
                    const double x = ci[3 * q], y = ci[3 * q + 1], z = ci[3 * q + 2];
                    for (int a = 0; a < 3; ++a) ci[3 * q + a] = T[a][0] * x + T[a][1] * y + T[a][2] * z;
                }
            }
        }
        coordmat.insert(coordmat.end(), ci.begin(), ci.end());
        for (long long v : P.elem) elementmat.push_back(v + nNode);
        nNode += P.nNode;
        nElement += P.nElement;
    }

    // ---- Amplitude (:624-668)
    std::vector<Amp> AMP;
    for (long long i = 1; i <= n; ++i) {
        if (!has(line(i), "*Amplitude")) continue;
        Amp a;
        auto ss = split(nospace(line(i)), ',', false);
        a.name = after(at(ss, 2), "name=");
        for (long long r = i + 1; r <= n; ++r) {
            if (has(line(r), "*")) break;
            auto t = split(nospace(line(r)), ',', false);
            if (t.size() % 2) throw ParseError{"InexactError: odd *Amplitude data line"};
            a.time.clear();
            a.value.clear();  // each data line replaces the table (reference quirk)
            for (size_t j = 0; j < t.size() / 2; ++j) {
                a.time.push_back(parse_f(t[2 * j]));
                a.value.push_back(parse_f(t[2 * j + 1]));
            }
        }
        AMP.push_back(a);
    }

    // ---- Material (:671-793)
    std::vector<long long> material_index;
    for (long long i = 1; i <= n; ++i)
        if (has(line(i), "*Material")) material_index.push_back(i);
    std::vector<Mat> MAT(material_index.size());
    for (size_t k = 0; k < MAT.size(); ++k) {
        Mat& m = MAT[k];
        auto ss = split(nospace(line(material_index[k])), ',', false);
        m.name = after(at(ss, 2), "name=");
        long long plastic_index = 1, ductile_index = 1;
        for (long long i = material_index[k] + 1; i <= n; ++i) {
            if (has(line(i), "*Material")) break;
            if (has(line(i), "**")) break;
            if (has(line(i), "*Density")) m.density = parse_f(at(split(nospace(line(i + 1)), ',', false), 1));
            if (has(line(i), "*Elastic")) {
                auto t = split(nospace(line(i + 1)), ',', false);
                m.young = parse_f(at(t, 1));
                m.poisson = parse_f(at(t, 2));
            }
            if (has(line(i), "*Plastic")) plastic_index = i;
            if (has(line(i), "*Damage Initiation") && has(line(i), "criterion=DUCTILE")) {
                ductile_index = i;
                m.fracture_flag = 1;
            }
            if (has(line(i), "*Tensile Failure")) {
                m.failure_stress = parse_f(at(split(nospace(line(i + 1)), ',', false), 1));
                m.fracture_flag = 1;
            }
        }
        if (plastic_index > material_index[k])
            for (long long i = plastic_index + 1; i <= n; ++i) {
                if (has(line(i), "*")) break;
                auto t = split(nospace(line(i)), ',', false);
                m.plastic.push_back(parse_f(at(t, 1)));
                m.plastic.push_back(parse_f(at(t, 2)));
            }
        if (ductile_index > material_index[k])
            for (long long i = ductile_index + 1; i <= n; ++i) {
                if (has(line(i), "*")) break;
                auto t = split(nospace(line(i)), ',', false);
                m.ductile.push_back(parse_f(at(t, 1)));
                m.ductile.push_back(parse_f(at(t, 2)));
                m.ductile.push_back(parse_f(at(t, 3)));
            }
    }

    // ---- element material / instance (:796-813)
    std::vector<long long> element_material, element_instance;
    for (size_t i = 0; i < INST.size(); ++i) {
        Part& P = PART[INST[i].part_id - 1];
        for (size_t j = 0; j < MAT.size(); ++j)
            if (P.material_name == MAT[j].name) {
                P.material_id = (int)j + 1;
                INST[i].material_id = (int)j + 1;
            }
        for (long long e = 0; e < P.nElement; ++e) {
            element_material.push_back(P.material_id);
            element_instance.push_back((long long)i + 1);
        }
    }

    // ---- Step / mass scaling (:816-840)
    double d_time = 0., end_time = 0.;
    for (long long i = 1; i <= n; ++i)
        if (has(line(i), "*Dynamic, Explicit")) {
            auto t = split(nospace(line(i + 1)), ',', false);
            d_time = parse_f(at(t, 1));
            end_time = parse_f(at(t, 2));
            break;
        }
    double mass_scaling = 1.;
    for (long long i = 1; i <= n; ++i)
        if (has(line(i), "*Fixed Mass Scaling")) {
            auto t = split(nospace(line(i)), ',', false);
            mass_scaling = parse_f(after(at(t, 2), "factor="));
            break;
        }

    // node-set resolution used by *Boundary / *Initial Conditions
    auto nodes_of = [&](const std::string& name, bool all_matches) {
        std::vector<long long> nodes;
        if (has(name, ".")) {
            auto sss = split(name, '.', false);
            const std::string inst = at(sss, 1), nset = at(sss, 2);
            int iid = 0, pid = 0;
            for (size_t j = 0; j < INST.size(); ++j)
                if (INST[j].name == inst) {
                    iid = (int)j + 1;
                    pid = INST[j].part_id;
                    break;
                }
            if (pid == 0) throw ParseError{"BoundsError: instance " + inst + " not found"};
            for (auto& ns : PART[pid - 1].nsets)
                if (ns.name == nset) {
                    for (long long v : ns.nodes) nodes.push_back(v + INST[iid - 1].node_offset);
                    break;
                }
        } else {
            for (auto& ns : NSET)
                if (ns.name == name) {
                    if (ns.instance_id == 0) throw ParseError{"BoundsError: nset instance not found"};
                    for (long long v : ns.nodes) nodes.push_back(v + INST[ns.instance_id - 1].node_offset);
                    if (!all_matches) break;
                }
        }
        return nodes;
    };

    // ---- Boundary (:843-957)
    std::vector<BC> BCS;
    for (long long bi = 1; bi <= n; ++bi) {
        if (!has(line(bi), "*Boundary")) continue;
        BC b;
        auto ss = split(nospace(line(bi)), ',', false);
        if (ss.size() == 2 && has(ss[1], "amplitude=")) {
            b.amp_name = after(ss[1], "amplitude=");
            for (auto& a : AMP)
                if (a.name == b.amp_name) {
                    b.amp = a;
                    break;
                }
        }
        for (long long i = bi + 1; i <= n; ++i) {
            if (has(line(i), "*Boundary")) break;
            if (has(line(i), "**")) break;
            auto t = split(nospace(line(i)), ',', false);
            const std::string nsn = at(t, 1);
            const std::vector<long long> nodes = nodes_of(nsn, true);
            if (t.size() == 2 && has(t[1], "ENCASTRE")) {
                std::vector<long long> dof;
                for (long long v : nodes) dof.push_back(v * 3 - 2);
                for (long long v : nodes) dof.push_back(v * 3 - 1);
                for (long long v : nodes) dof.push_back(v * 3);
                b.dof.push_back(dof);
                b.value.assign(1, 0.);
            } else if (t.size() == 3) {
                (void)parse_i(t[1]);
                const long long dir = parse_i(t[2]);
                if (dir <= 3) {
                    std::vector<long long> dof;
                    for (long long v : nodes) dof.push_back(v * 3 - (3 - dir));
                    b.dof.push_back(dof);
                    b.value.push_back(0.);
                }
            } else if (t.size() == 4) {
                (void)parse_i(t[1]);
                const long long dir = parse_i(t[2]);
                const double value = parse_f(t[3]);
                if (dir <= 3) {
                    std::vector<long long> dof;
                    for (long long v : nodes) dof.push_back(v * 3 - (3 - dir));
                    b.dof.push_back(dof);
                    b.value.push_back(value);
                }
            }
        }
        if (b.value.size() < b.dof.size())
            throw ParseError{"BoundsError: *Boundary block mixes ENCASTRE with other lines (v2/HAKAI_j.jl:607)"};
        BCS.push_back(b);
    }

    // ---- Initial Conditions (:960-1043)
    std::vector<IC> ICS;
    for (long long ii = 1; ii <= n; ++ii) {
        if (!has(line(ii), "*Initial Conditions")) continue;
        IC c;
        auto ss = split(nospace(line(ii)), ',', false);
        (void)after(at(ss, 2), "type=");
        for (long long i = ii + 1; i <= n; ++i) {
            if (has(line(i), "*Initial Conditions")) break;
            if (has(line(i), "**")) break;
            auto t = split(nospace(line(i)), ',', false);
            const std::vector<long long> nodes = nodes_of(at(t, 1), false);
            const long long dir = parse_i(at(t, 2));
            const double v = parse_f(at(t, 3));
            std::vector<long long> dof;
            for (long long q : nodes) dof.push_back(q * 3 - (3 - dir));
            c.dof.push_back(dof);
            c.value.push_back(v);
        }
        ICS.push_back(c);
    }

    // ---- contact flags (:1046-1060)
    int contact_flag = 0;
    for (long long i = 1; i <= n; ++i)
        if (has(line(i), "*Contact")) {
            contact_flag = 1;
            break;
        }
    for (long long i = 1; i <= n; ++i)
        if (has(line(i), "*Contact Inclusions") && has(line(i), "HAKAIoption=self-contact")) {
            contact_flag = 2;
            break;
        }
    // ---- *Surface (:517-564): element sets (face ids ignored), instance of the last listed elset
    struct Surf {
        std::string name;
        int instance_id = 0;
        std::vector<long long> elements;
    };
    std::vector<Surf> SURF;
    for (long long i = 1; i <= n; ++i) {
        if (!has(line(i), "*Surface,")) continue;
        Surf sf;
        sf.name = after(at(split(nospace(line(i)), ',', false), 3), "name=");
        for (long long r = i + 1; r <= n; ++r) {
            if (has(line(r), "*")) break;
            const std::string es = at(split(nospace(line(r)), ',', false), 1);
            for (auto& E : ELSET)
                if (E.name == es) {
                    sf.instance_id = E.instance_id;
                    sf.elements.insert(sf.elements.end(), E.elements.begin(), E.elements.end());
                }
        }
        std::sort(sf.elements.begin(), sf.elements.end());
        sf.elements.erase(std::unique(sf.elements.begin(), sf.elements.end()), sf.elements.end());
        SURF.push_back(sf);
    }
    // ---- *Contact Pair (:1063-1102): the two surfaces on the line after the keyword
    o.cp_inst.clear();
    o.cp_off.assign(1, 0);
    o.cp_elems.clear();
    for (long long i = 1; i <= n; ++i) {
        if (!has(line(i), "*Contact Pair,")) continue;
        const auto names = split(nospace(line(i + 1)), ',', false);
        for (int s = 0; s < 2; ++s) {
            const std::string& nm = at(names, s + 1);
            const Surf* hit = nullptr;
            for (auto& sf : SURF)
                if (sf.name == nm) hit = &sf;
            if (!hit || hit->instance_id == 0) throw ParseError{"*Contact Pair: unknown surface " + nm};
            o.cp_inst.push_back(hit->instance_id);
            o.cp_elems.insert(o.cp_elems.end(), hit->elements.begin(), hit->elements.end());
            o.cp_off.push_back((int64_t)o.cp_elems.size());
        }
    }

    // ---- flatten into the C view
    o.coord = coordmat;
    o.elem.assign(elementmat.begin(), elementmat.end());
    o.emat.assign(element_material.begin(), element_material.end());
    o.einst.assign(element_instance.begin(), element_instance.end());
    o.mat_pl.resize(MAT.size());
    o.mat_du.resize(MAT.size());
    o.mats.resize(MAT.size());
    for (size_t k = 0; k < MAT.size(); ++k) {
        o.mat_pl[k] = MAT[k].plastic;
        o.mat_du[k] = MAT[k].ductile;
        hakai_material_t& hm = o.mats[k];
        hm.density = MAT[k].density;
        hm.young = MAT[k].young;
        hm.poisson = MAT[k].poisson;
        hm.n_plastic = (int32_t)(MAT[k].plastic.size() / 2);
        hm.plastic = o.mat_pl[k].data();
        hm.n_ductile = (int32_t)(MAT[k].ductile.size() / 3);
        hm.ductile = o.mat_du[k].data();
    }
    for (auto& b : BCS) {
        o.amp_off.push_back((int64_t)o.amp_t.size());
        if (b.amp_name.empty()) {
            o.amp_n.push_back(0);
        } else {
            o.amp_n.push_back((int32_t)b.amp.time.size());
            o.amp_t.insert(o.amp_t.end(), b.amp.time.begin(), b.amp.time.end());
            o.amp_v.insert(o.amp_v.end(), b.amp.value.begin(), b.amp.value.end());
        }
        o.entry_off.push_back((int64_t)o.entry_val.size());
        for (size_t j = 0; j < b.dof.size(); ++j) {
            o.dof_off.push_back((int64_t)o.dofs.size());
            o.entry_val.push_back(b.value[j]);
            for (long long d : b.dof[j]) o.dofs.push_back(d);
        }
    }
    o.entry_off.push_back((int64_t)o.entry_val.size());
    o.dof_off.push_back((int64_t)o.dofs.size());
    for (auto& c : ICS)
        for (size_t j = 0; j < c.dof.size(); ++j)
            for (long long d : c.dof[j]) {
                o.ic_dofs.push_back(d);
                o.ic_val.push_back(c.value[j]);
            }
    for (auto& I : INST) {
        o.inst_noff.push_back(I.node_offset);
        o.inst_eoff.push_back(I.element_offset);
        o.inst_ne.push_back(I.nElement);
    }
    hakai_inp_model_t& p = o.pub;
    std::memset(&p, 0, sizeof p);
    p.nNode = nNode;
    p.coordmat = o.coord.data();
    p.nElement = nElement;
    p.elementmat = o.elem.data();
    p.element_material = o.emat.data();
    p.element_instance = o.einst.data();
    p.nMat = (int32_t)o.mats.size();
    p.materials = o.mats.data();
    p.d_time = d_time;
    p.end_time = end_time;
    p.mass_scaling = mass_scaling;
    p.contact_flag = contact_flag;
    p.n_cp = (int32_t)o.cp_inst.size() / 2;
    p.cp_instance = o.cp_inst.data();
    p.cp_elem_off = o.cp_off.data();
    p.cp_elems = o.cp_elems.data();
    p.bc.n_groups = (int32_t)BCS.size();
    p.bc.amp_n = o.amp_n.data();
    p.bc.amp_off = o.amp_off.data();
    p.bc.amp_time = o.amp_t.data();
    p.bc.amp_value = o.amp_v.data();
    p.bc.entry_off = o.entry_off.data();
    p.bc.entry_value = o.entry_val.data();
    p.bc.dof_off = o.dof_off.data();
    p.bc.dofs = o.dofs.data();
    p.n_ic_dofs = (int64_t)o.ic_dofs.size();
    p.ic_dofs = o.ic_dofs.data();
    p.ic_values = o.ic_val.data();
    p.n_instance = (int32_t)INST.size();
    p.instance_node_offset = o.inst_noff.data();
    p.instance_element_offset = o.inst_eoff.data();
    p.instance_nElement = o.inst_ne.data();
}

void pusai_table(double P[8][3][8]) {  // cal_Pusai_hexa, v2/HAKAI_j.jl:1895-1943
    static const double delta[8][3] = {{-1.0, -1.0, -1.0}, {1.0, -1.0, -1.0}, {1.0, 1.0, -1.0}, {-1.0, 1.0, -1.0},
                                       {-1.0, -1.0, 1.0},  {1.0, -1.0, 1.0},  {1.0, 1.0, 1.0},  {-1.0, 1.0, 1.0}};
    const double g = 1.0 / std::sqrt(3.0);
    const double gc[8][3] = {{-g, -g, -g}, {-g, -g, g}, {-g, g, -g}, {-g, g, g},
                             {g, -g, -g},  {g, -g, g},  {g, g, -g},  {g, g, g}};
    for (int k = 0; k < 8; ++k)
        for (int i = 0; i < 8; ++i) {
            P[k][0][i] = 1.0 / 8.0 * delta[i][0] * (1.0 + gc[k][1] * delta[i][1]) * (1.0 + gc[k][2] * delta[i][2]);
            P[k][1][i] = 1.0 / 8.0 * delta[i][1] * (1.0 + gc[k][0] * delta[i][0]) * (1.0 + gc[k][2] * delta[i][2]);
            P[k][2][i] = 1.0 / 8.0 * delta[i][2] * (1.0 + gc[k][0] * delta[i][0]) * (1.0 + gc[k][1] * delta[i][1]);
        }
}

}  // namespace

extern "C" {

int hakai_inp_read(const char* path, hakai_inp_model_t** out) {
    if (!path || !out) return fail(HAKAI_ERR_ARG, "null");
    *out = nullptr;
    std::unique_ptr<Owned> o(new Owned());
    try {
        parse(path, *o);
    } catch (const ParseError& e) {
        return fail(HAKAI_ERR_IO, "%s: %s", path, e.msg.c_str());
    } catch (const std::exception& e) {
        return fail(HAKAI_ERR_IO, "%s: %s", path, e.what());
    }
    *out = &o.release()->pub;
    return 0;
}

void hakai_inp_free(hakai_inp_model_t* m) {
    if (!m) return;
    delete reinterpret_cast<Owned*>(m);  // pub is the first member
}

int hakai_lumped_mass(int64_t nNode, const double* coordmat, int64_t nElement, const int64_t* elementmat,
                      const int64_t* element_material, int32_t nMat, const hakai_material_t* mats, double mass_scaling,
                      double* diag_M, double* elementVolume) {

    if (nNode <= 0 || nElement < 0 || !coordmat || !diag_M || (nElement > 0 && (!elementmat || !element_material)))
        return fail(HAKAI_ERR_ARG, "lumped_mass: bad arguments");
    double P[8][3][8];
    pusai_table(P);
    std::vector<double> vol((size_t)nElement);
    for (int64_t e = 0; e < nElement; ++e) {
        double X[3][8];
        for (int i = 0; i < 8; ++i) {
            const int64_t nn = elementmat[8 * e + i] - 1;
            if (nn < 0 || nn >= nNode) return fail(HAKAI_ERR_ARG, "lumped_mass: node index out of range");
            for (int c = 0; c < 3; ++c) X[c][i] = coordmat[3 * nn + c];
        }
        double V = 0.;
        for (int k = 0; k < 8; ++k) {
            double J[3][3];
            for (int a = 0; a < 3; ++a)
                for (int b = 0; b < 3; ++b) {
                    double acc = P[k][a][0] * X[b][0];
                    for (int i = 1; i < 8; ++i) acc = acc + P[k][a][i] * X[b][i];
                    J[a][b] = acc;
                }
            V = V + (J[0][0] * J[1][1] * J[2][2] + J[0][1] * J[1][2] * J[2][0] + J[0][2] * J[1][0] * J[2][1] -
                     J[0][0] * J[1][2] * J[2][1] - J[0][1] * J[1][0] * J[2][2] - J[0][2] * J[1][1] * J[2][0]);
        }
        vol[e] = V;
    }
    for (int64_t i = 0; i < 3 * nNode; ++i) diag_M[i] = 0.0;
    for (int64_t e = 0; e < nElement; ++e) {
        const int64_t m = element_material[e];
        if (m < 1 || m > nMat) return fail(HAKAI_ERR_ARG, "lumped_mass: material index out of range");
        const double node_mass = mats[m - 1].density * vol[e] / 8.0;
        for (int c = 0; c < 3; ++c)
            for (int i = 0; i < 8; ++i) diag_M[(elementmat[8 * e + i] - 1) * 3 + c] += node_mass;
    }
    for (int64_t i = 0; i < 3 * nNode; ++i) diag_M[i] = diag_M[i] * mass_scaling;
    if (elementVolume)
        for (int64_t e = 0; e < nElement; ++e) elementVolume[e] = vol[e];
    return 0;
}

int hakai_run_inp(const char* fname, const char* out_dir, int device, int verbose) {
    hakai_inp_model_t* M = nullptr;
    int r = hakai_inp_read(fname, &M);
    if (r) return r;
    struct FreeM {
        hakai_inp_model_t* m;
        ~FreeM() { hakai_inp_free(m); }
    } fm{M};
    if (verbose) {
        std::printf("readInpFile:%s\n", fname);
        std::printf("nNode:%lld\nnElement:%lld\ncontact_flag:%d\n", (long long)M->nNode, (long long)M->nElement,
                    M->contact_flag);
    }
    const long long nN = M->nNode, nE = M->nElement;
    const double d_time = M->d_time * std::sqrt(M->mass_scaling);  // v2/HAKAI_j.jl:114
    const double time_num = M->end_time / d_time;
    if (verbose) std::printf("mass_scaling:%g\ntime_num:%g\n", M->mass_scaling, time_num);
    std::vector<double> diag_M(3 * (size_t)nN);
    r = hakai_lumped_mass(nN, M->coordmat, nE, M->elementmat, M->element_material, M->nMat, M->materials,
                          M->mass_scaling, diag_M.data(), nullptr);
    if (r) return r;
    hakai_ctx* c = nullptr;
    r = hakai_create(&c, device);
    if (r) return r;
    struct FreeC {
        hakai_ctx* c;
        ~FreeC() { hakai_destroy(c); }
    } fc{c};
    // The driver reproduces the reference's element arithmetic operation for operation
    // (elem_exact), so its output is the reference's bits; HAKAI_ELEM_EXACT=0 selects the fused
    // single-pass kernel (same physics, rounding-level differences).
    const char* ex = std::getenv("HAKAI_ELEM_EXACT");
    if ((r = hakai_set_tuning(c, "elem_exact", (ex && ex[0] == '0') ? 0 : 1))) return r;
    if ((r = hakai_upload_model(c, nN, M->coordmat, nE, M->elementmat, M->element_material, M->nMat, M->materials,
                                diag_M.data())))
        return r;
    if ((r = hakai_set_bc(c, &M->bc))) return r;
    if (M->contact_flag >= 1 && (r = hakai_set_contact_cp(c, M->contact_flag, M->element_instance, M->n_cp,
                                                          M->cp_instance, M->cp_elem_off, M->cp_elems)))
        return r;
    if ((r = hakai_reset_state(c, M->n_ic_dofs, M->ic_dofs, M->ic_values, d_time))) return r;
    const long long n_steps = time_num >= 1.0 ? (long long)std::floor(time_num) : 0;
    const long long d_out = (long long)std::floor(time_num / 100);  // output_num = 100 (:471-472)
    // VTK files are formatted and written by the writer's thread team while the device steps on;
    // the arrays go straight from the device into the writer's fill buffers (zero-copy commit).
    const char* se = std::getenv("HAKAI_VTK_SYNC");  // 1: wait for every file (A/B measurements)
    const bool sync_out = se && se[0] == '1';
    hakai_vtk_writer* w = nullptr;
    if ((r = hakai_vtk_writer_create(&w, out_dir, nN, M->coordmat, nE, M->elementmat, 0))) return r;
    struct FreeW {
        hakai_vtk_writer* w;
        ~FreeW() { hakai_vtk_writer_destroy(w); }
    } fw{w};
    auto output = [&](int idx) -> int {
        hakai_vtk_arrays_t a;
        int q = hakai_vtk_writer_acquire(w, &a);
        if (q) return q;
        hakai_state_t st;
        std::memset(&st, 0, sizeof st);
        st.disp = a.disp;
        st.velo = a.velo;
        st.element_flag = a.element_flag;
        if ((q = hakai_download_state(c, &st))) return q;
        if ((q = hakai_node_stress_strain(c, a.node_stress, a.node_strain, a.node_eq_plastic_strain,
                                          a.node_mises_stress, a.node_triax_stress)))
            return q;
        if ((q = hakai_vtk_writer_commit(w, idx))) return q;
        return sync_out ? hakai_vtk_writer_wait(w) : 0;
    };
    if ((r = output(0))) return r;
    int i_out = 1;
    long long t0 = 1, reported = 0;
    while (t0 <= n_steps) {
        long long t1 = n_steps;
        if (d_out > 0) t1 = std::min(n_steps, ((t0 + d_out - 1) / d_out) * d_out);
        if ((r = hakai_step(c, (double)t0, t1 - t0 + 1, d_time))) return r;
        if (verbose) {
            int64_t nd = 0;
            hakai_deleted(c, &nd, nullptr, 0);
            for (long long q = reported; q < nd; ++q)
                std::printf("Element deleted:%lld/%lld\n", (long long)(nE - q - 1), nE);
            reported = nd;
            std::printf("\r%.4e / %.4e     ", (double)t1 * d_time, M->end_time);
            std::fflush(stdout);
        }
        if (d_out > 0 && t1 % d_out == 0) {
            if ((r = output(i_out))) return r;
            ++i_out;
        }
        t0 = t1 + 1;
    }
    if ((r = hakai_sync(c))) return r;
    if ((r = hakai_vtk_writer_wait(w))) return r;
    if (verbose) std::printf("\n");
    return 0;
}

}  // extern "C"
