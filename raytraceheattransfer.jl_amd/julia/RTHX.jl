"""
    RTHX

Julia `ccall` shim that routes RayTraceHeatTransfer.jl's exchange-factor
tracer (`mesh(N_rays; method=:exchange)`) to the MI355X kernels of
`librthx.so` (C ABI: `include/rthx.h`).

The seam is `computeExchangeFactorsBin`
(src/RayTracing/RayTracing2D/ExchangeFactors2D/parallelRayTracing.jl:64-159);
everything above it (bin grouping, surfaces-only truncation, `smooth_F`,
`solveEquilibrium!`) is unchanged.  Usage:

    using RayTraceHeatTransfer
    include("raytraceheattransfer.jl_amd/julia/RTHX.jl")
    RTHX.enable!(; lib = "raytraceheattransfer.jl_amd/csrc/_build/librthx.so", device = 0, seed = 1)
    mesh(100_000_000; method = :exchange)      # traced on the GPU
    RTHX.enable!(; lib = ..., devices = 0:7)   # rows split over 8 GPUs (rthx_multi_trace_exchange)

Not executable in the build container (no Julia toolchain); kept in step
with `include/rthx.h` by `tests/test_abi.py::test_julia_shim_mirrors_header`.
"""
module RTHX

using SparseArrays

const RTHX_ABI_VERSION = Int32(3)
const RTHX_FLAG_FAITHFUL_SAMPLING = UInt32(0x1)

const LIB = Ref{String}("")
const DEVICE = Ref{Int32}(0)          # device of the single-device calls (first of DEVICES)
const DEVICES = Ref{Vector{Int32}}(Int32[0])  # devices the exchange tracer splits its rows over
const SEED = Ref{UInt64}(1)
const FAITHFUL = Ref{Bool}(false)

# --- C structs (field order and types exactly as include/rthx.h) ----------
struct GridDesc
    origin_x::Float64
    origin_y::Float64
    inv_cell_size::Float64
    nx::Int32
    ny::Int32
    cell_start::Ptr{Int32}
    cell_items::Ptr{Int32}
end

struct DomainDesc
    abi_version::Int32
    n_coarse::Int32
    n_fine::Int32
    n_surfaces::Int32
    n_bins::Int32
    reserved0::Int32
    coarse_nv::Ptr{Int32}
    coarse_xy::Ptr{Float64}
    coarse_normal::Ptr{Float64}
    coarse_solid::Ptr{UInt8}
    coarse_bbox::Ptr{Float64}
    coarse_grid::GridDesc
    fine_offset::Ptr{Int32}
    fine_nv::Ptr{Int32}
    fine_xy::Ptr{Float64}
    fine_normal::Ptr{Float64}
    fine_mid::Ptr{Float64}
    fine_volume::Ptr{Float64}
    fine_bbox::Ptr{Float64}
    fine_surface::Ptr{Int32}
    fine_grid::Ptr{GridDesc}
    beta::Ptr{Float64}
    uniform_beta::Ptr{Float64}
end

struct TraceArgs
    bin::Int32
    flags::UInt32
    rays_per_emitter::Int64
    nudge::Float64
    seed::UInt64
    emitter_begin::Int64
    emitter_end::Int64
    emitter_stride::Int64
    device::Int32
    n_record::Int32
    record_ids::Ptr{Int64}
    record_bin::Int32
    reserved0::Int32
end

struct ResultInfo
    n_emitters::Int64
    rows_traced::Int64
    rays_per_emitter::Int64
    rays_traced::Int64
    nnz::Int64
    lost_total::Int64
    lost_max_row::Int64
    n_recorded::Int64
    trace_ms::Float64
    pack_ms::Float64
    total_ms::Float64
    n_devices::Int32
    lookback_fallbacks::Int32
    superseded::Int32
    superseded_faults::Int32
end

struct SmoothArgs
    device::Int32
    max_iters::Int32
    k_dykstra::Int32
    smooth_surfaces_only::Int32
    renorm::Int32
    verbose::Int32
    input_dense::Int32
    reserved0::Int32
end

struct SmoothInfo
    n::Int64
    nnz::Int64
    dense::Int32
    k_dykstra::Int32
    pcg_iters::Int32
    ap_iters::Int32
    converged::Int32
    floor_accepted::Int32
    chi::Float64
    delta_init::Float64
    delta_final::Float64
    ms_op::Float64
    ms_ap::Float64
    ms_total::Float64
end

struct DirectArgs
    rays::Int64
    ray_begin::Int64
    ray_end::Int64
    nudge::Float64
    seed::UInt64
    bin::Int32
    device::Int32
    max_iters::Int32
    roulette_after::Int32
    roulette_kill::Float64
    flags::UInt32
    reserved0::Int32
end

struct DirectInfo
    rays_traced::Int64
    absorbed::Int64
    escaped::Int64
    rouletted::Int64
    capped::Int64
    events::Int64
    replayed::Int64
    trace_ms::Float64
    total_ms::Float64
end

struct Vf3dArgs
    device::Int32
    reserved0::Int32
end

struct Vf3dInfo
    n::Int64
    pairs::Int64
    kernel_ms::Float64
    total_ms::Float64
end

function check(rc::Integer)
    if rc != 0
        msg = unsafe_string(ccall((:rthx_last_error, LIB[]), Cstring, ()))
        error("rthx error $rc: $msg")
    end
end

# --- flattening RayTracingDomain2D (DomainStructs.jl:89-130) --------------
"Host arrays of one flattened domain; kept alive while the descriptor is used."
mutable struct Flat
    arrays::Vector{Any}
    grids::Vector{GridDesc}
    desc::Base.RefValue{DomainDesc}
end

function grid_arrays(g)  # UniformGrid (DomainStructs.jl:79-86): cells[i, j] lists face indices
    nx, ny = g.nx, g.ny
    start = zeros(Int32, nx * ny + 1)
    items = Int32[]
    for j in 1:ny, i in 1:nx
        for f in g.cells[i, j]
            push!(items, Int32(f - 1))
        end
        start[(j - 1) * nx + i + 1] = length(items)
    end
    isempty(items) && push!(items, Int32(0))
    return start, items
end

polyxy(p) = (v = zeros(Float64, 8); for (k, q) in enumerate(p.vertices); v[2k-1] = q[1]; v[2k] = q[2]; end;
             length(p.vertices) == 3 && (v[7] = v[5]; v[8] = v[6]); v)
polynrm(p) = (v = zeros(Float64, 8); for (k, q) in enumerate(p.inwardNormals); v[2k-1] = q[1]; v[2k] = q[2]; end; v)
bbox(p) = (xs = [q[1] for q in p.vertices]; ys = [q[2] for q in p.vertices];
           [minimum(xs), maximum(xs), minimum(ys), maximum(ys)])
betaof(f, b) = f.kappa_g isa AbstractVector ? f.kappa_g[b] + f.sigma_s_g[b] : f.kappa_g + f.sigma_s_g

function flatten(rtm)
    coarse = rtm.coarse_mesh
    fine = rtm.fine_mesh
    nc = length(coarse)
    offs = Int32[0; cumsum([Int32(length(s)) for s in fine])]
    faces = [f for s in fine for f in s]
    nf = length(faces)
    ns = length(rtm.surface_mapping)
    nb = rtm.n_spectral_bins
    c_nv = Int32[length(c.vertices) for c in coarse]
    c_xy = reduce(vcat, [polyxy(c) for c in coarse])
    c_n = reduce(vcat, [polynrm(c) for c in coarse])
    c_s = reduce(vcat, [UInt8[(k <= length(c.solidWalls) && c.solidWalls[k]) for k in 1:4] for c in coarse])
    c_bb = reduce(vcat, [bbox(c) for c in coarse])
    f_nv = Int32[length(f.vertices) for f in faces]
    f_xy = reduce(vcat, [polyxy(f) for f in faces])
    f_n = reduce(vcat, [polynrm(f) for f in faces])
    f_mid = reduce(vcat, [[f.midPoint[1], f.midPoint[2]] for f in faces])
    f_vol = Float64[f.volume for f in faces]
    f_bb = reduce(vcat, [bbox(f) for f in faces])
    f_surf = fill(Int32(-1), 4 * nf)
    for ((c, f, w), s) in rtm.surface_mapping
        f_surf[4 * (offs[c] + f - 1) + w] = Int32(s - 1)
    end
    beta = Float64[betaof(faces[k], b) for k in 1:nf, b in 1:nb][:]  # [bin][face] (column-major = bin-major)
    ub = Float64.(rtm.uniform_across_bin)
    cg_start, cg_items = grid_arrays(rtm.coarse_grid_opt)
    keep = Any[c_nv, c_xy, c_n, c_s, c_bb, f_nv, f_xy, f_n, f_mid, f_vol, f_bb, f_surf, beta, ub, offs,
               cg_start, cg_items]
    mk(g, st, it) = GridDesc(g.origin[1], g.origin[2], g.inv_cell_size, Int32(g.nx), Int32(g.ny),
                             pointer(st), pointer(it))
    grids = GridDesc[]
    for c in 1:nc
        st, it = grid_arrays(rtm.fine_grids_opt[c])
        push!(keep, st, it)
        push!(grids, mk(rtm.fine_grids_opt[c], st, it))
    end
    push!(keep, grids)
    desc = DomainDesc(RTHX_ABI_VERSION, Int32(nc), Int32(nf), Int32(ns), Int32(nb), Int32(0),
                      pointer(c_nv), pointer(c_xy), pointer(c_n), pointer(c_s), pointer(c_bb),
                      mk(rtm.coarse_grid_opt, cg_start, cg_items),
                      pointer(offs), pointer(f_nv), pointer(f_xy), pointer(f_n), pointer(f_mid), pointer(f_vol),
                      pointer(f_bb), pointer(f_surf), pointer(grids), pointer(beta), pointer(ub))
    return Flat(keep, grids, Ref(desc))
end

# --- uploaded domains -------------------------------------------------------
# One upload per (rtm, kind): an rthx_domain (one device) or an rthx_multi
# (DEVICES, rows split over them).  The reference reads the domain live at
# every trace (traceRay.jl:87-100 reads kappa_g / sigma_s_g per segment, and
# its tests set n_spectral_bins after construction, test/test_2d_spectral.jl:79),
# so every call flattens rtm again and compares the flattened geometry,
# beta[fine, bin] and uniform_across_bin with the upload's (same_domain): a
# mutated domain, another device list or another library is uploaded again.
# Uploads are held in a WeakKeyDict (rtm is a mutable struct): when rtm is
# collected the entry goes, and the Uploaded's finalizer frees the device
# copy.  `invalidate!(rtm)` and `release_all!()` free them explicitly.
mutable struct Uploaded
    flat::Flat
    handle::Ptr{Cvoid}
    multi::Bool
    devices::Vector{Int32}
    lib::String
end

function release!(u::Uploaded)
    if u.handle != C_NULL
        ccall((u.multi ? :rthx_multi_destroy : :rthx_domain_destroy, u.lib), Cvoid, (Ptr{Cvoid},), u.handle)
        u.handle = C_NULL
    end
    return nothing
end

const UPLOADS = WeakKeyDict{Any, Dict{Bool, Uploaded}}()

"""
    same_domain(a::Flat, b::Flat)

Element-wise equality of two flattenings' numeric arrays (geometry, grids,
LUTs, beta[fine, bin], uniform_across_bin), not of their descriptors, whose
pointers differ per flatten.  (Base's `hash` of a large array samples only
some elements, so a changed kappa could hash alike: compare them all.)
"""
same_domain(a::Flat, b::Flat) =
    length(a.arrays) == length(b.arrays) &&
    all(x isa Vector{GridDesc} || isequal(x, y) for (x, y) in zip(a.arrays, b.arrays))

"""
    invalidate!(rtm)

Free rtm's uploaded device copies (both kinds); the next trace uploads it
again.  Mutations are also caught by the per-call comparison.
"""
function invalidate!(rtm)
    ups = pop!(UPLOADS, rtm, nothing)
    ups === nothing || foreach(release!, values(ups))
    return nothing
end

"Free every uploaded domain (e.g. before `enable!` with another library)."
function release_all!()
    for k in collect(keys(UPLOADS))
        invalidate!(k)
    end
    return nothing
end

function uploaded(rtm, multi::Bool)
    flat = flatten(rtm)
    devs = multi ? copy(DEVICES[]) : Int32[DEVICE[]]
    ups = get!(() -> Dict{Bool, Uploaded}(), UPLOADS, rtm)
    u = get(ups, multi, nothing)
    if u !== nothing && u.handle != C_NULL && same_domain(u.flat, flat) && u.devices == devs && u.lib == LIB[]
        return u.handle
    end
    u === nothing || release!(u)
    h = Ref{Ptr{Cvoid}}(C_NULL)
    GC.@preserve flat devs begin
        if multi
            check(ccall((:rthx_multi_create, LIB[]), Cint, (Ptr{DomainDesc}, Ptr{Int32}, Int32, Ptr{Ptr{Cvoid}}),
                        flat.desc, devs, Int32(length(devs)), h))
        else
            check(ccall((:rthx_domain_create, LIB[]), Cint, (Ptr{DomainDesc}, Int32, Ptr{Ptr{Cvoid}}),
                        flat.desc, devs[1], h))
        end
    end
    u = Uploaded(flat, h[], multi, devs, LIB[])
    finalizer(release!, u)
    ups[multi] = u
    return u.handle
end

device_domain(rtm) = uploaded(rtm, false)
multi_domain(rtm) = uploaded(rtm, true)

"""
    computeExchangeFactorsBin(rtm, rays_per_emitter, nudge, spectral_bin, surface_mapping,
                              volume_mapping, num_surfaces, num_volumes, num_emitters, verbose, rec)

Drop-in for parallelRayTracing.jl:64-159: one `rthx_trace_exchange` call,
then F_raw (the reference's `sparse` + `row_normalize!`, :154-169) formed
and laid out as SparseMatrixCSC on the device (`rthx_result_copy_F_csc`).
"""
function computeExchangeFactorsBin(rtm, rays_per_emitter::Integer, nudge, spectral_bin::Integer,
                                   surface_mapping, volume_mapping, num_surfaces, num_volumes, num_emitters,
                                   verbose, rec)
    multi = length(DEVICES[]) > 1
    dom = multi ? multi_domain(rtm) : device_domain(rtm)
    ids = rec === nothing ? Int64[] : Int64[i - 1 for i in rec.ids]
    rbin = rec === nothing ? Int32(0) : Int32(rec.bin - 1)
    args = Ref(TraceArgs(Int32(spectral_bin - 1), FAITHFUL[] ? RTHX_FLAG_FAITHFUL_SAMPLING : UInt32(0),
                         Int64(rays_per_emitter), Float64(nudge), SEED[], 0, Int64(num_emitters), 1, DEVICE[],
                         Int32(length(ids)), isempty(ids) ? Ptr{Int64}(C_NULL) : pointer(ids), rbin, Int32(0)))
    res = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:rthx_result_create, LIB[]), Cint, (Ptr{Ptr{Cvoid}},), res))
    try
        GC.@preserve ids begin
            check(ccall((multi ? :rthx_multi_trace_exchange : :rthx_trace_exchange, LIB[]), Cint,
                        (Ptr{Cvoid}, Ptr{TraceArgs}, Ptr{Cvoid}), dom, args, res[]))
        end
        info = Ref{ResultInfo}()
        check(ccall((:rthx_result_get_info, LIB[]), Cint, (Ptr{Cvoid}, Ptr{ResultInfo}), res[], info))
        N, nnz = info[].n_emitters, info[].nnz
        # F_raw in Julia's own CSC layout (1-based), formed and transposed on
        # the device: no host transpose of the CSR (at C2, 3e7 nonzeros)
        colptr = Vector{Int64}(undef, N + 1)
        rowval = Vector{Int64}(undef, nnz)
        nzval = Vector{Float64}(undef, nnz)
        check(ccall((:rthx_result_copy_F_csc, LIB[]), Cint, (Ptr{Cvoid}, Int32, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}),
                    res[], Int32(1), colptr, rowval, nzval))
        verbose && println("  rthx: $(info[].rays_traced) rays on $(info[].n_devices) device(s), nnz $nnz, ",
                           "trace $(round(info[].trace_ms; digits=3)) ms")
        if rec !== nothing && info[].n_recorded > 0
            n = info[].n_recorded
            o = Vector{Float64}(undef, 2n); e = Vector{Float64}(undef, 2n); g = Vector{Int64}(undef, n)
            nout = Ref{Int64}(0)
            check(ccall((:rthx_result_copy_rays, LIB[]), Cint,
                        (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Int64}, Int64, Ptr{Int64}),
                        res[], o, e, g, n, nout))
            for k in 1:nout[]
                push!(rec.origins[1], eltype(rec.origins[1])(o[2k-1], o[2k]))
                push!(rec.endpoints[1], eltype(rec.endpoints[1])(e[2k-1], e[2k]))
            end
        end
        # The reference's sparse(I, J, V) + row_normalize! (parallelRayTracing.jl:154-169):
        # every row divided by its sum, here count / (rays the row tallied) on the
        # device, and row_normalize!'s loss line from the trace's lost-ray count
        # (R * max|1 - row sum| = the most rays one row lost, :163)
        println("Maximum ray tracing ray loss per emitter: $(info[].lost_max_row)/$rays_per_emitter")
        return SparseMatrixCSC(N, N, colptr, rowval, nzval)
    finally
        ccall((:rthx_result_destroy, LIB[]), Cvoid, (Ptr{Cvoid},), res[])
    end
end

"""
    smooth_F(F_raw, w, num_surfaces; max_iters=1000, smooth_surfaces_only=false,
             k_dykstra=nothing, verbose=true, renorm=true)

Device smoothing with the signature and result kind of the reference's
smooth_F (smoothExchangeFactors.jl:412-459): a dense Matrix when it smooths
densely, a SparseMatrixCSC otherwise.
"""
function smooth_F(F_raw::AbstractMatrix, w::AbstractVector, num_surfaces::Integer; max_iters::Integer = 1000,
                  smooth_surfaces_only::Bool = false, k_dykstra = nothing, verbose::Bool = true,
                  renorm::Bool = true)
    input_dense = !(F_raw isa SparseMatrixCSC)
    Fr = SparseMatrixCSC(transpose(sparse(F_raw)))      # CSC of F' = CSR of F
    n = size(F_raw, 1)
    rowptr = Int64.(Fr.colptr) .- 1
    cols = Int32.(Fr.rowval) .- Int32(1)
    vals = Vector{Float64}(Fr.nzval)
    ww = Vector{Float64}(w)
    args = Ref(SmoothArgs(DEVICE[], Int32(max_iters), Int32(k_dykstra === nothing ? -1 : k_dykstra),
                          Int32(smooth_surfaces_only), Int32(renorm), Int32(verbose), Int32(input_dense), Int32(0)))
    h = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:rthx_smooth_F, LIB[]), Cint,
                (Ptr{Int64}, Ptr{Int32}, Ptr{Float64}, Int64, Ptr{Float64}, Int64, Int32, Ptr{SmoothArgs},
                 Ptr{Ptr{Cvoid}}),
                rowptr, cols, vals, n, ww, length(ww), Int32(num_surfaces), args, h))
    try
        info = Ref{SmoothInfo}()
        check(ccall((:rthx_smooth_get_info, LIB[]), Cint, (Ptr{Cvoid}, Ptr{SmoothInfo}), h[], info))
        m = info[].n
        if info[].dense == 1
            out = Matrix{Float64}(undef, m, m)   # row-major from the library = transpose in Julia
            check(ccall((:rthx_smooth_copy_dense, LIB[]), Cint, (Ptr{Cvoid}, Ptr{Float64}), h[], out))
            return permutedims(out)
        else
            nnz = info[].nnz
            rp = Vector{Int64}(undef, m + 1); ci = Vector{Int32}(undef, max(nnz, 1)); v = Vector{Float64}(undef, max(nnz, 1))
            check(ccall((:rthx_smooth_copy_csr, LIB[]), Cint, (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int32}, Ptr{Float64}),
                        h[], rp, ci, v))
            Ft = SparseMatrixCSC(m, m, rp .+ 1, Int64.(ci[1:nnz]) .+ 1, v[1:nnz])
            return SparseMatrixCSC(transpose(Ft))
        end
    finally
        ccall((:rthx_smooth_destroy, LIB[]), Cvoid, (Ptr{Cvoid},), h[])
    end
end

"""
    directRayTracingSingleBin!(rtm, rays_tot, nudge, spectral_bin)

Drop-in for directRayTracing.jl:19-152: the reference's prepareEmitters gives
the energies; the ray loop (:69-128, traceSingleRay) is one
`rthx_trace_direct` call; the counts go back into the reference's nested
counter arrays and through its own updateSpectralResults! (:148-151).
"""
function directRayTracingSingleBin!(rtm, rays_tot::Integer, nudge, spectral_bin::Integer)
    RTHT = parentmodule(@__MODULE__).RayTraceHeatTransfer
    emitters, total_energy = RTHT.prepareEmitters(rtm, nudge, spectral_bin)
    if total_energy == 0.0
        @warn "No emitters found for spectral bin $spectral_bin, skipping ray tracing"
        return
    end
    Ns = length(rtm.surface_mapping)
    n = Ns + length(rtm.volume_mapping)
    w = zeros(Float64, n); eps = zeros(Float64, max(Ns, 1)); omega = zeros(Float64, n - Ns); reemit = zeros(UInt8, n)
    for e in emitters  # energies in global element order (getGlobalIndex2D.jl:1-15)
        g = e.type == :surface ? rtm.surface_mapping[(e.coarse_index, e.fine_index, e.wall_index)] :
                                 Ns + rtm.volume_mapping[(e.coarse_index, e.fine_index)]
        w[g] = e.energy
    end
    pick(v, b) = v isa AbstractVector ? v[b] : v
    for ((c, f, k), s) in rtm.surface_mapping
        face = rtm.fine_mesh[c][f]
        eps[s] = pick(face.epsilon[k], spectral_bin)
        reemit[s] = face.T_in_w[k] < 0.0
    end
    for ((c, f), v) in rtm.volume_mapping
        face = rtm.fine_mesh[c][f]
        kap = pick(face.kappa_g, spectral_bin); sig = pick(face.sigma_s_g, spectral_bin)
        omega[v] = kap + sig != 0 ? sig / (kap + sig) : 0.0
        reemit[Ns + v] = face.T_in_g < 0.0
    end
    args = Ref(DirectArgs(Int64(rays_tot), 0, Int64(rays_tot), Float64(nudge), SEED[], Int32(spectral_bin - 1),
                          DEVICE[], Int32(100_000), Int32(1000), 0.8,
                          FAITHFUL[] ? RTHX_FLAG_FAITHFUL_SAMPLING : UInt32(0), Int32(0)))
    counts = zeros(UInt64, 3n)
    info = Ref{DirectInfo}()
    check(ccall((:rthx_trace_direct, LIB[]), Cint,
                (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ptr{UInt8}, Ptr{DirectArgs}, Ptr{UInt64},
                 Ptr{DirectInfo}),
                device_domain(rtm), w, eps, omega, reemit, args, counts, info))
    # back into the reference's counters (directRayTracing.jl:29-34)
    cm = rtm.coarse_mesh
    absorbed = [zeros(Int, length(cf.subVolumes)) for cf in cm]
    gas_emitted = [zeros(Int, length(cf.subVolumes)) for cf in cm]
    scattered = [zeros(Int, length(cf.subVolumes)) for cf in cm]
    wall_emitted = [[zeros(Int, length(f.solidWalls)) for f in cf.subVolumes] for cf in cm]
    reflected = [[zeros(Int, length(f.solidWalls)) for f in cf.subVolumes] for cf in cm]
    wall_absorbed = [[zeros(Int, length(f.solidWalls)) for f in cf.subVolumes] for cf in cm]
    for ((c, f, k), s) in rtm.surface_mapping
        wall_emitted[c][f][k] = counts[s]; wall_absorbed[c][f][k] = counts[n + s]; reflected[c][f][k] = counts[2n + s]
    end
    for ((c, f), v) in rtm.volume_mapping
        g = Ns + v
        gas_emitted[c][f] = counts[g]; absorbed[c][f] = counts[n + g]; scattered[c][f] = counts[2n + g]
    end
    RTHT.updateSpectralResults!(rtm, absorbed, gas_emitted, wall_emitted, reflected, scattered, wall_absorbed,
                                total_energy, rays_tot, spectral_bin)
    return nothing
end

"""
    enclosureViewFactors3D(superFaces, parallel, max_iters=1000)

Drop-in for enclosureViewFactors3D.jl:1-94: every ordered sub-face pair's
viewFactor3D on the device (`rthx_view_factors_3d`, sub-faces in the
reference's face-major linear order, fromLinear :96-100), areas written back
to the sub-faces (:48-49), then the reference's own smooth_F with
smooth_surfaces_only = true (:88-91).
"""
function enclosureViewFactors3D(superFaces, parallel::Bool, max_iters::Int = 1000)
    RTHT = parentmodule(@__MODULE__).RayTraceHeatTransfer
    subs = [sf for f in superFaces for sf in f.subFaces]
    n = length(subs)
    xyz = zeros(Float64, 12n); nv = zeros(Int32, n)
    for (k, sf) in enumerate(subs)
        nv[k] = length(sf.vertices)
        for (i, v) in enumerate(sf.vertices), d in 1:3
            xyz[12(k - 1) + 3(i - 1) + d] = v[d]
        end
    end
    Ft = Matrix{Float64}(undef, n, n)      # row-major from the library = F' in Julia's layout
    area = Vector{Float64}(undef, n)
    info = Ref{Vf3dInfo}()
    args = Ref(Vf3dArgs(DEVICE[], Int32(0)))
    check(ccall((:rthx_view_factors_3d, LIB[]), Cint,
                (Ptr{Float64}, Ptr{Int32}, Int64, Ptr{Vf3dArgs}, Ptr{Float64}, Ptr{Float64}, Ptr{Vf3dInfo}),
                xyz, nv, n, args, Ft, area, info))
    F_raw = permutedims(Ft)
    for (k, sf) in enumerate(subs)
        sf.area = area[k]
    end
    F_smooth = RTHT.smooth_F(F_raw, area, n; max_iters = max_iters, smooth_surfaces_only = true)
    return F_raw, F_smooth
end

"""
    enclosureViewFactorsMC3D(superFaces, rays_tot; max_iters=1000)

Monte Carlo counterpart of enclosureViewFactors3D for enclosures with
obstructions (BASELINE config 4: a sphere inside a cube), where the analytic
pair view factors (which assume every pair sees each other) do not hold.
Sub-faces in the same face-major order; each leaves along its inwardNormal,
and the sub-faces of one super face form a coplanar group (a ray is never
absorbed by its own face).
`rays_tot` rays in total, div(rays_tot, n) per sub-face as the 2D tracer
(parallelRayTracing.jl:6).  F_raw = counts / R, row-normalised like the 2D
path (row_normalize!), then the reference's smooth_F with
smooth_surfaces_only = true (enclosureViewFactors3D.jl:88-91).
"""
function enclosureViewFactorsMC3D(superFaces, rays_tot::Integer; max_iters::Int = 1000, verbose::Bool = false)
    RTHT = parentmodule(@__MODULE__).RayTraceHeatTransfer
    subs = [sf for f in superFaces for sf in f.subFaces]
    # the sub-faces of one super face are coplanar: one group (contiguous, face-major)
    grp = Int32[i - 1 for (i, f) in enumerate(superFaces) for _ in f.subFaces]
    n = length(subs)
    xyz = zeros(Float64, 12n); nv = zeros(Int32, n); nrm = zeros(Float64, 3n)
    for (k, sf) in enumerate(subs)
        nv[k] = length(sf.vertices)
        for (i, v) in enumerate(sf.vertices), d in 1:3
            xyz[12(k - 1) + 3(i - 1) + d] = v[d]
        end
        for d in 1:3
            nrm[3(k - 1) + d] = sf.inwardNormal[d]
        end
    end
    R = div(rays_tot, n)
    scene = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:rthx_scene3d_create_grouped, LIB[]), Cint,
                (Ptr{Float64}, Ptr{Int32}, Ptr{Float64}, Ptr{Int32}, Int64, Int32, Ptr{Ptr{Cvoid}}),
                xyz, nv, nrm, grp, n, DEVICE[], scene))
    res = Ref{Ptr{Cvoid}}(C_NULL)
    try
        check(ccall((:rthx_result_create, LIB[]), Cint, (Ptr{Ptr{Cvoid}},), res))
        args = Ref(TraceArgs(Int32(0), FAITHFUL[] ? RTHX_FLAG_FAITHFUL_SAMPLING : UInt32(0), Int64(R), 0.0,
                             SEED[], 0, Int64(n), 1, DEVICE[], Int32(0), Ptr{Int64}(C_NULL), Int32(0), Int32(0)))
        check(ccall((:rthx_trace_exchange_3d, LIB[]), Cint, (Ptr{Cvoid}, Ptr{TraceArgs}, Ptr{Cvoid}),
                    scene[], args, res[]))
        info = Ref{ResultInfo}()
        check(ccall((:rthx_result_get_info, LIB[]), Cint, (Ptr{Cvoid}, Ptr{ResultInfo}), res[], info))
        nnz = info[].nnz
        rowptr = Vector{Int64}(undef, n + 1)
        cols = Vector{Int32}(undef, max(nnz, 1))
        counts = Vector{UInt32}(undef, max(nnz, 1))
        check(ccall((:rthx_result_copy_csr, LIB[]), Cint, (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int32}, Ptr{UInt32}),
                    res[], rowptr, cols, counts))
        verbose && println("  rthx 3D: $(info[].rays_traced) rays, lost $(info[].lost_total), trace $(round(info[].trace_ms; digits=3)) ms")
        Ft = SparseMatrixCSC(n, n, rowptr .+ 1, Int64.(cols[1:nnz]) .+ 1, Float64.(counts[1:nnz]) ./ R)
        F_raw = Matrix(transpose(Ft))
        F_raw = Matrix(RTHT.row_normalize!(sparse(F_raw), R))
        # polygon areas as viewFactor3D.jl:47-76 (triangle |n|/2, quad |(P3-P1) x (P4-P2)|/2), written
        # back to the sub-faces like enclosureViewFactors3D.jl:48-49
        cr(a, b) = (a[2]b[3] - a[3]b[2], a[3]b[1] - a[1]b[3], a[1]b[2] - a[2]b[1])
        nrm2(v) = sqrt(v[1]^2 + v[2]^2 + v[3]^2)
        area = map(subs) do sf
            P = sf.vertices
            length(P) == 3 ? nrm2(cr(P[2] .- P[1], P[3] .- P[1])) / 2 : nrm2(cr(P[3] .- P[1], P[4] .- P[2])) / 2
        end
        for (k, sf) in enumerate(subs)
            sf.area = area[k]
        end
        F_smooth = RTHT.smooth_F(F_raw, area, n; max_iters = max_iters, smooth_surfaces_only = true)
        return F_raw, F_smooth
    finally
        res[] != C_NULL && ccall((:rthx_result_destroy, LIB[]), Cvoid, (Ptr{Cvoid},), res[])
        ccall((:rthx_scene3d_destroy, LIB[]), Cvoid, (Ptr{Cvoid},), scene[])
    end
end

"""
    enable!(; lib, device=0, devices=[device], seed=1, faithful=false)

Redirect RayTraceHeatTransfer's `computeExchangeFactorsBin` (and, with
`direct = true`, `directRayTracingSingleBin!`; with `viewfactors3d = true`,
`enclosureViewFactors3D`) to the GPU.  With several `devices` the exchange
tracer splits each bin's emitter rows over them (rthx_multi_trace_exchange:
one host thread and stream per GPU, the counts identical to one device's);
the other calls run on the first.
"""
function enable!(; lib::AbstractString, device::Integer = 0, devices = [device], seed::Integer = 1,
                 faithful::Bool = false, smoothing::Bool = false, direct::Bool = true, viewfactors3d::Bool = true)
    lib == LIB[] || release_all!()  # (uploads belong to the library that made them)
    LIB[] = lib
    DEVICES[] = Int32[d for d in devices]
    isempty(DEVICES[]) && error("enable!: empty device list")
    DEVICE[] = DEVICES[][1]
    SEED[] = UInt64(seed)
    FAITHFUL[] = faithful
    v = ccall((:rthx_abi_version, LIB[]), Cint, ())
    v == RTHX_ABI_VERSION || error("librthx ABI $v, shim expects $RTHX_ABI_VERSION")
    RTHT = parentmodule(@__MODULE__).RayTraceHeatTransfer
    @eval RTHT function computeExchangeFactorsBin(rtm::RayTracingDomain2D, rays_per_emitter::P, nudge::G,
                                                  spectral_bin::P, surface_mapping, volume_mapping,
                                                  num_surfaces, num_volumes, num_emitters, verbose,
                                                  rec) where {P<:Integer, G}
        return $(RTHX).computeExchangeFactorsBin(rtm, rays_per_emitter, nudge, spectral_bin, surface_mapping,
                                                 volume_mapping, num_surfaces, num_volumes, num_emitters,
                                                 verbose, rec)
    end
    if viewfactors3d  # 3D enclosures: analytic view factors on the device
        @eval RTHT function enclosureViewFactors3D(superFaces::Vector{PolyFace3D{G}}, parallel::Bool,
                                                  max_iters::Int = 1000) where G
            return $(RTHX).enclosureViewFactors3D(superFaces, parallel, max_iters)
        end
    end
    if direct  # method=:direct on the device as well
        @eval RTHT function directRayTracingSingleBin!(rtm::RayTracingDomain2D, rays_tot::P, nudge::G,
                                                      spectral_bin::P) where {G, P<:Integer}
            return $(RTHX).directRayTracingSingleBin!(rtm, rays_tot, nudge, spectral_bin)
        end
    end
    if smoothing  # optional: smooth_F on the device as well
        @eval RTHT function smooth_F(F_raw::AbstractMatrix, w::AbstractVector, num_surfaces::Int; kw...)
            return $(RTHX).smooth_F(F_raw, w, num_surfaces; kw...)
        end
    end
    return nothing
end

end # module
