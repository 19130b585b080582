# HakaiHIP.jl -- ccall layer over libhakai_hip.so for HAKAI v0.0.2 (yozoyugen/HAKAI-fem).
#
# What a HAKAI maintainer adds next to HAKAI-v0.0.2/Julia/HAKAI_j.jl:
#     include("HakaiHIP.jl")            # after include("./readInpFile_j.jl") and HAKAI_j.jl's types
#     HakaiHIP.hakai_gpu("deck.inp")    # = hakai(fname) (v2/HAKAI_j.jl:81-978) with the time loop on the GPU
# Every ccall below is checked against include/hakai_hip.h by tests/test_julia_shim.py (argument
# count and C <-> Julia type of every argument and struct field). Julia is not installed in the
# build container or on the GPU box, so this file has never been executed.
#
# Conventions (SURVEY.md §10): the reference's own arrays are passed as they are -- Float64,
# Int64 1-based indices, column-major (coordmat 3 x nNode, elementmat 8 x nElement, integ_stress
# 6 x 8nElement, Qe 24 x nElement). The library converts layouts and never keeps Julia memory.
module HakaiHIP

using Printf

const lib = get(ENV, "HAKAI_HIP_LIB", joinpath(@__DIR__, "..", "hakai-fem_amd", "lib", "libhakai_hip.so"))

# ---- C structs (include/hakai_hip.h) -----------------------------------------------------------
struct Material            # hakai_material_t (MaterialType, v2/readInpFile_j.jl:84-96)
    density::Float64
    young::Float64
    poisson::Float64
    n_plastic::Int32
    plastic::Ptr{Float64}  # row-major [n_plastic][2]
    n_ductile::Int32
    ductile::Ptr{Float64}  # row-major [n_ductile][3]
end

struct BC                  # hakai_bc_t (the BCType list, v2/readInpFile_j.jl:98-104)
    n_groups::Int32
    amp_n::Ptr{Int32}
    amp_off::Ptr{Int64}
    amp_time::Ptr{Float64}
    amp_value::Ptr{Float64}
    entry_off::Ptr{Int64}
    entry_value::Ptr{Float64}
    dof_off::Ptr{Int64}
    dofs::Ptr{Int64}
end

struct State               # hakai_state_t; C_NULL skips an array
    disp::Ptr{Float64}
    disp_pre::Ptr{Float64}
    velo::Ptr{Float64}
    Q::Ptr{Float64}
    integ_stress::Ptr{Float64}
    integ_strain::Ptr{Float64}
    integ_yield_stress::Ptr{Float64}
    integ_eq_plastic_strain::Ptr{Float64}
    integ_triax_stress::Ptr{Float64}
    element_flag::Ptr{Int64}
    Qe::Ptr{Float64}
end

check(rc) = rc == 0 || error("libhakai_hip: ", unsafe_string(ccall((:hakai_last_error, lib), Cstring, ())))
abi_version() = ccall((:hakai_abi_version, lib), Cint, ())
function device_count()
    n = Ref{Cint}(0)
    check(ccall((:hakai_device_count, lib), Cint, (Ref{Cint},), n))
    return n[]
end

# MaterialType -> hakai_material_t; the ABI wants row-major plastic/ductile tables: permuted
# copies, kept alive by the caller (GC.@preserve keep)
function materials(MATERIAL)
    keep = Any[]
    mats = Material[]
    for m in MATERIAL
        p = Matrix{Float64}(permutedims(m.plastic)); d = Matrix{Float64}(permutedims(m.ductile))
        push!(keep, p, d)
        push!(mats, Material(m.density, m.young, m.poisson, size(m.plastic, 1), pointer(p),
                             size(m.ductile, 1), pointer(d)))
    end
    return mats, keep
end

# ---- context (replaces hakai()'s state, v2/HAKAI_j.jl:81-480) -----------------------------------
mutable struct Ctx
    p::Ptr{Cvoid}
end
function create(device::Integer = 0)
    r = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:hakai_create, lib), Cint, (Ref{Ptr{Cvoid}}, Cint), r, device))
    c = Ctx(r[])
    finalizer(destroy, c)
    return c
end
destroy(c::Ctx) = (c.p != C_NULL && ccall((:hakai_destroy, lib), Cint, (Ptr{Cvoid},), c.p); c.p = C_NULL; nothing)

function upload_model(c::Ctx, coordmat, elementmat, element_material, MATERIAL, diag_M)
    mats, keep = materials(MATERIAL)
    GC.@preserve keep mats check(ccall((:hakai_upload_model, lib), Cint,
        (Ptr{Cvoid}, Int64, Ptr{Float64}, Int64, Ptr{Int64}, Ptr{Int64}, Int32, Ptr{Material}, Ptr{Float64}),
        c.p, size(coordmat, 2), coordmat, size(elementmat, 2), elementmat, element_material,
        length(mats), mats, diag_M))
end

# MODEL.BC (v2/HAKAI_j.jl:585-617: groups in order, entries (dof list, value), amplitude by name)
function set_bc(c::Ctx, BCs)
    amp_n = Int32[]; amp_off = Int64[]; amp_t = Float64[]; amp_v = Float64[]
    entry_off = Int64[0]; entry_value = Float64[]; dof_off = Int64[0]; dofs = Int64[]
    for b in BCs
        if length(b.amp_name) > 0
            push!(amp_n, length(b.amplitude.time)); push!(amp_off, length(amp_t))
            append!(amp_t, b.amplitude.time); append!(amp_v, b.amplitude.value)
        else
            push!(amp_n, 0); push!(amp_off, length(amp_t))
        end
        for j = 1:length(b.dof)
            push!(entry_value, b.value[j]); append!(dofs, b.dof[j]); push!(dof_off, length(dofs))
        end
        push!(entry_off, length(entry_value))
    end
    GC.@preserve amp_n amp_off amp_t amp_v entry_off entry_value dof_off dofs begin
        bc = Ref(BC(length(BCs), pointer(amp_n), pointer(amp_off), pointer(amp_t), pointer(amp_v),
                    pointer(entry_off), pointer(entry_value), pointer(dof_off), pointer(dofs)))
        check(ccall((:hakai_set_bc, lib), Cint, (Ptr{Cvoid}, Ref{BC}), c.p, bc))
    end
end

# fresh state + MODEL.IC velocities (v2/HAKAI_j.jl:225-239, :430-465)
function reset_state(c::Ctx, ICs, d_time)
    ic_dofs = Int64[]; ic_values = Float64[]
    for ic in ICs, j = 1:length(ic.dof)
        append!(ic_dofs, ic.dof[j]); append!(ic_values, fill(ic.value[j], length(ic.dof[j])))
    end
    check(ccall((:hakai_reset_state, lib), Cint, (Ptr{Cvoid}, Int64, Ptr{Int64}, Ptr{Float64}, Float64),
                c.p, length(ic_dofs), ic_dofs, ic_values, d_time))
end

_p(a) = a === nothing ? C_NULL : pointer(a)
function state(; disp = nothing, disp_pre = nothing, velo = nothing, Q = nothing, integ_stress = nothing,
               integ_strain = nothing, integ_yield_stress = nothing, integ_eq_plastic_strain = nothing,
               integ_triax_stress = nothing, element_flag = nothing, Qe = nothing)
    return State(_p(disp), _p(disp_pre), _p(velo), _p(Q), _p(integ_stress), _p(integ_strain),
                 _p(integ_yield_stress), _p(integ_eq_plastic_strain), _p(integ_triax_stress),
                 _p(element_flag), _p(Qe))
end
# the arrays named in kw are filled in place (same layout as the reference's; velo = d_disp/d_time)
function download_state!(c::Ctx; kw...)
    arrays = values(kw)
    GC.@preserve arrays check(ccall((:hakai_download_state, lib), Cint, (Ptr{Cvoid}, Ref{State}), c.p,
                                    Ref(state(; kw...))))
end
function upload_state(c::Ctx; kw...)
    arrays = values(kw)
    GC.@preserve arrays check(ccall((:hakai_upload_state, lib), Cint, (Ptr{Cvoid}, Ref{State}), c.p,
                                    Ref(state(; kw...))))
end

# n iterations of the loop body v2/HAKAI_j.jl:497-764 for t = t_first .. t_first+n-1
step!(c::Ctx, t_first, n, d_time) =
    check(ccall((:hakai_step, lib), Cint, (Ptr{Cvoid}, Float64, Int64, Float64), c.p, t_first, n, d_time))
sync(c::Ctx) = check(ccall((:hakai_sync, lib), Cint, (Ptr{Cvoid},), c.p))
# an in-process group (rank r = cs[r+1]) in lockstep: every rank's contact phases A1, A2, A3, then
# every rank's event sums, exchange and update, per step (multi-GPU contact in one process)
function step_group!(cs::Vector{Ctx}, t_first, n, d_time)
    ps = Ptr{Cvoid}[c.p for c in cs]
    check(ccall((:hakai_step_group, lib), Cint, (Ptr{Ptr{Cvoid}}, Int32, Float64, Int64, Float64), ps,
                length(cs), t_first, n, d_time))
end
function graph_steps(c::Ctx)
    n = Ref{Int64}(0)
    check(ccall((:hakai_graph_steps, lib), Cint, (Ptr{Cvoid}, Ref{Int64}), c.p, n))
    return n[]
end
# step-loop counters: "graph_steps", "own_steps", "own_rows", "own_entries", "own_superbatch", "own_slots"
function stat(c::Ctx, key::AbstractString)
    n = Ref{Int64}(0)
    check(ccall((:hakai_stat, lib), Cint, (Ptr{Cvoid}, Cstring, Ref{Int64}), c.p, key, n))
    return n[]
end
# (step, element) of every deletion so far, in the order the reference prints them (:733-736)
function deleted(c::Ctx; cap::Integer = 1 << 16)
    n = Ref{Int64}(0)
    log = zeros(Int64, 2, cap)
    check(ccall((:hakai_deleted, lib), Cint, (Ptr{Cvoid}, Ref{Int64}, Ptr{Int64}, Int64), c.p, n, log, cap))
    return log[:, 1:min(n[], cap)]
end
function negative_jacobians(c::Ctx)
    n = Ref{Int64}(0)
    check(ccall((:hakai_negative_jacobians, lib), Cint, (Ptr{Cvoid}, Ref{Int64}), c.p, n))
    return n[]
end
set_tuning(c::Ctx, key::AbstractString, value::Integer) =
    check(ccall((:hakai_set_tuning, lib), Cint, (Ptr{Cvoid}, Cstring, Int64), c.p, key, value))

# cal_node_stress_strain (v2/HAKAI_j.jl:3408-3486) on the device -> the fields of NodeDataType
# (node_stress / node_strain nNode x 6 like the reference; node_plastic_strain stays zero, :450)
function node_stress_strain(c::Ctx, nNode::Integer)
    ns = zeros(6, nNode); nn = zeros(6, nNode)
    ne = zeros(nNode); nm = zeros(nNode); nt = zeros(nNode)
    check(ccall((:hakai_node_stress_strain, lib), Cint,
                (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                c.p, ns, nn, ne, nm, nt))
    return (node_stress = permutedims(ns), node_strain = permutedims(nn), node_plastic_strain = zeros(nNode, 6),
            node_eq_plastic_strain = ne, node_mises_stress = nm, node_triax_stress = nt)
end

# ---- literal drop-ins ----------------------------------------------------------------------
# v2/HAKAI_j.jl:664-667 (def :1033-1036): same arrays, mutated in place (PCIe-bound: for parity)
function cal_stress_hexa(Qe, integ_stress, integ_strain, integ_yield_stress, integ_eq_plastic_strain,
                         position, d_disp, elementmat, element_flag, integ_num, Pusai_mat, MATERIAL,
                         element_material, elementMinSize, elementVolume; device::Integer = 0)
    mats, keep = materials(MATERIAL)
    GC.@preserve keep mats check(ccall((:hakai_stress_hexa, lib), Cint,
        (Cint, Int64, Int64, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
         Ptr{Float64}, Ptr{Float64}, Ptr{Int64}, Ptr{Int64}, Int32, Int32, Ptr{Material}, Ptr{Int64},
         Ptr{Float64}),
        device, size(position, 2), size(elementmat, 2), Qe, integ_stress, integ_strain,
        integ_yield_stress, integ_eq_plastic_strain, position, d_disp, elementmat, element_flag,
        integ_num, length(mats), mats, element_material, elementVolume))
    return nothing
end
# v2/HAKAI_j.jl:677 (def :982)
cal_triax_stress(integ_stress, integ_triax_stress; device::Integer = 0) =
    check(ccall((:hakai_triax_stress, lib), Cint, (Cint, Int64, Ptr{Float64}, Ptr{Float64}),
                device, size(integ_stress, 2), integ_stress, integ_triax_stress))
# v2/HAKAI_j.jl:183-218 (host only)
function lumped_mass(coordmat, elementmat, element_material, MATERIAL, mass_scaling)
    mats, keep = materials(MATERIAL)
    diag_M = zeros(3 * size(coordmat, 2)); vol = zeros(size(elementmat, 2))
    GC.@preserve keep mats check(ccall((:hakai_lumped_mass, lib), Cint,
        (Int64, Ptr{Float64}, Int64, Ptr{Int64}, Ptr{Int64}, Int32, Ptr{Material}, Float64, Ptr{Float64},
         Ptr{Float64}),
        size(coordmat, 2), coordmat, size(elementmat, 2), elementmat, element_material, length(mats), mats,
        mass_scaling, diag_M, vol))
    return diag_M, vol
end

# ---- contact (v2/HAKAI_j.jl:244-421 setup, :500-560 per step, :766-804 surface update) ----------
set_contact(c::Ctx, contact_flag, element_instance::Vector{Int64}) =
    check(ccall((:hakai_set_contact, lib), Cint, (Ptr{Cvoid}, Int32, Ptr{Int64}), c.p, contact_flag, element_instance))
# *Contact Pair decks: MODEL.CP (v2/readInpFile_j.jl:1063-1102), surfaces as instance-local elements
function set_contact_cp(c::Ctx, contact_flag, element_instance::Vector{Int64}, CPs)
    cp_instance = Int32[]; cp_elem_off = Int64[0]; cp_elems = Int64[]
    for cp in CPs
        push!(cp_instance, cp.instance_id_1, cp.instance_id_2)
        append!(cp_elems, cp.elements_1); push!(cp_elem_off, length(cp_elems))
        append!(cp_elems, cp.elements_2); push!(cp_elem_off, length(cp_elems))
    end
    check(ccall((:hakai_set_contact_cp, lib), Cint,
                (Ptr{Cvoid}, Int32, Ptr{Int64}, Int32, Ptr{Int32}, Ptr{Int64}, Ptr{Int64}),
                c.p, contact_flag, element_instance, length(CPs), cp_instance, cp_elem_off, cp_elems))
end
set_contact_params(c::Ctx; myu = 0.25, kc_o = 1.0, kc_s = 1.0, Cr_o = 0.0, Cr_s = 0.0) =
    check(ccall((:hakai_set_contact_params, lib), Cint, (Ptr{Cvoid}, Float64, Float64, Float64, Float64, Float64),
                c.p, myu, kc_o, kc_s, Cr_o, Cr_s))
contact_force!(c::Ctx, external_force, t, d_time) =
    check(ccall((:hakai_contact_force, lib), Cint, (Ptr{Cvoid}, Float64, Float64, Ptr{Float64}),
                c.p, t, d_time, external_force))
function contact_stats(c::Ctx)
    st = zeros(Int64, 10)
    check(ccall((:hakai_contact_stats, lib), Cint, (Ptr{Cvoid}, Ptr{Int64}, Int32), c.p, st, length(st)))
    return st
end

# ---- multi-GPU (one Julia process per GPU; see INTEGRATION.md) ----------------------------------
function comm_unique_id()
    id = zeros(UInt8, 128)
    check(ccall((:hakai_comm_unique_id, lib), Cint, (Ptr{UInt8},), id))
    return id
end
comm_init(c::Ctx, rank, nranks, id::Vector{UInt8}) =
    check(ccall((:hakai_comm_init, lib), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{UInt8}), c.p, rank, nranks, id))
# an in-process group of contexts on one device (rank r of n, same key on every member)
comm_init_local(c::Ctx, rank, nranks, key) =
    check(ccall((:hakai_comm_init_local, lib), Cint, (Ptr{Cvoid}, Cint, Cint, Int64), c.p, rank, nranks, key))
set_interface(c::Ctx, local_node::Vector{Int64}, rank_lo::Vector{Int32}, rank_hi::Vector{Int32}) =
    check(ccall((:hakai_set_interface, lib), Cint, (Ptr{Cvoid}, Int64, Ptr{Int64}, Ptr{Int32}, Ptr{Int32}),
                c.p, length(local_node), local_node, rank_lo, rank_hi))
set_element_offset(c::Ctx, offset) =
    check(ccall((:hakai_set_element_offset, lib), Cint, (Ptr{Cvoid}, Int64), c.p, offset))

# multi-GPU contact: every rank passes the GLOBAL contact model (arguments as hakai_upload_model /
# set_contact_cp for the whole mesh) plus its local->global node map and the ranks' element ranges;
# it keeps its own triangles and contact nodes (owner-computed search)
function set_contact_global(c::Ctx, contact_flag, coordmat, elementmat, element_material,
                            element_instance::Vector{Int64}, diag_M, local_node_global::Vector{Int64},
                            rank_elem_off::Vector{Int64}, CPs)
    cp_instance = Int32[]; cp_elem_off = Int64[0]; cp_elems = Int64[]
    for cp in CPs
        push!(cp_instance, cp.instance_id_1, cp.instance_id_2)
        append!(cp_elems, cp.elements_1); push!(cp_elem_off, length(cp_elems))
        append!(cp_elems, cp.elements_2); push!(cp_elem_off, length(cp_elems))
    end
    check(ccall((:hakai_set_contact_global, lib), Cint,
                (Ptr{Cvoid}, Int32, Int64, Ptr{Float64}, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Int64}, Ptr{Float64},
                 Ptr{Int64}, Ptr{Int64}, Int32, Ptr{Int32}, Ptr{Int64}, Ptr{Int64}),
                c.p, contact_flag, size(coordmat, 2), coordmat, size(elementmat, 2), elementmat, element_material,
                element_instance, diag_M, local_node_global, rank_elem_off, length(CPs), cp_instance, cp_elem_off,
                cp_elems))
end

# ---- per-kernel device time (HIP events on the context's stream) ----------------------------------
const K_ELEMENT, K_NODAL, K_BC, K_EXCHANGE, K_CONTACT = 0, 1, 2, 3, 4
profile(c::Ctx, on::Bool) = check(ccall((:hakai_profile_enable, lib), Cint, (Ptr{Cvoid}, Cint), c.p, on))
function profile_read(c::Ctx, kernel::Integer)
    ms = Ref{Float64}(0.0); n = Ref{Int64}(0)
    check(ccall((:hakai_profile_read, lib), Cint, (Ptr{Cvoid}, Cint, Ref{Float64}, Ref{Int64}), c.p, kernel, ms, n))
    return ms[], n[]
end

# ---- output: the library's asynchronous VTK writer (same bytes as write_vtk, :3517-3717) --------
mutable struct VtkWriter
    p::Ptr{Cvoid}
end
function vtk_writer(dir, coordmat, elementmat; threads::Integer = 0)
    w = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:hakai_vtk_writer_create, lib), Cint,
                (Ref{Ptr{Cvoid}}, Cstring, Int64, Ptr{Float64}, Int64, Ptr{Int64}, Cint),
                w, dir, size(coordmat, 2), coordmat, size(elementmat, 2), elementmat, threads))
    return VtkWriter(w[])
end
vtk_submit(w::VtkWriter, index, element_flag, disp, velo, nd) =
    check(ccall((:hakai_vtk_writer_submit, lib), Cint,
                (Ptr{Cvoid}, Cint, Ptr{Int64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64},
                 Ptr{Float64}, Ptr{Float64}, Ptr{Float64}),
                w.p, index, element_flag, disp, velo, permutedims(nd.node_stress), permutedims(nd.node_strain),
                nd.node_eq_plastic_strain, nd.node_mises_stress, nd.node_triax_stress))
vtk_wait(w::VtkWriter) = check(ccall((:hakai_vtk_writer_wait, lib), Cint, (Ptr{Cvoid},), w.p))
vtk_close(w::VtkWriter) = (ccall((:hakai_vtk_writer_destroy, lib), Cvoid, (Ptr{Cvoid},), w.p); w.p = C_NULL)

# ---- HAKAI(fname) with the loop body on the GPU ---------------------------------------------------
# The reference's own reader (readInpFile, v2/readInpFile_j.jl:152) and, by default, its own
# write_vtk (v2/HAKAI_j.jl:3517); `writer = true` uses the library's asynchronous writer instead.
# elem_exact = 1 (the default): the element update follows cal_stress_hexa's arithmetic operation for
# operation, so the run is the reference's bit for bit (tests/test_gpu_exact.py).
function hakai_gpu(fname; device::Integer = 0, writer::Bool = false, elem_exact::Integer = 1)
    MODEL = Main.readInpFile(fname)
    nNode, nElement = MODEL.nNode, MODEL.nElement
    coordmat, elementmat = MODEL.coordmat, MODEL.elementmat
    d_time = MODEL.d_time * sqrt(MODEL.mass_scaling)                  # :114
    time_num = MODEL.end_time / d_time
    diag_M, _ = lumped_mass(coordmat, elementmat, MODEL.element_material, MODEL.MATERIAL, MODEL.mass_scaling)
    c = create(device)
    set_tuning(c, "elem_exact", elem_exact)
    upload_model(c, coordmat, elementmat, MODEL.element_material, MODEL.MATERIAL, diag_M)
    set_bc(c, MODEL.BC)
    if MODEL.contact_flag >= 1
        set_contact_cp(c, MODEL.contact_flag, Vector{Int64}(MODEL.element_instance), MODEL.CP)
    end
    reset_state(c, MODEL.IC, d_time)
    fn = 3 * nNode
    disp = zeros(fn); velo = zeros(fn); element_flag = ones(Int64, nElement)
    w = writer ? vtk_writer("temp", coordmat, elementmat) : nothing
    function output(i_out)                                               # :932-942
        download_state!(c; disp = disp, velo = velo, element_flag = element_flag)
        nd = node_stress_strain(c, nNode)
        if writer
            vtk_submit(w, i_out, element_flag, disp, velo, nd)
        else
            node_data = Main.NodeDataType(nd.node_stress, nd.node_strain, nd.node_plastic_strain,
                                          nd.node_eq_plastic_strain, nd.node_mises_stress, nd.node_triax_stress)
            Main.write_vtk(i_out, coordmat, elementmat, element_flag, disp, copy(velo), node_data)
        end
    end
    output(0)
    d_out = Int(floor(time_num / 100))                                   # :471-472
    n_steps = Int(floor(time_num))
    reported = 0
    t0 = 1
    while t0 <= n_steps
        t1 = d_out > 0 ? min(n_steps, cld(t0, d_out) * d_out) : n_steps
        step!(c, t0, t1 - t0 + 1, d_time)
        dl = deleted(c)
        for q = reported+1:size(dl, 2)                                   # :736
            println("Element deleted:", nElement - q, "/", nElement)
        end
        reported = size(dl, 2)
        print(@sprintf("\r%.4e / %.4e     ", t1 * d_time, MODEL.end_time))
        if d_out > 0 && t1 % d_out == 0
            output(t1 ÷ d_out)
        end
        t0 = t1 + 1
    end
    sync(c)
    writer && (vtk_wait(w); vtk_close(w))
    println("")
    return nothing
end

# The driver surface in one call (reader, setup, loop, VTK all inside the library): v2/HAKAI_j.jl:81
run_inp(fname; out_dir = "temp", device = 0, verbose = 1) =
    check(ccall((:hakai_run_inp, lib), Cint, (Cstring, Cstring, Cint, Cint), fname, out_dir, device, verbose))

end # module
