# SCSOptAMD.jl -- Julia `ccall` binding of libscsopt (include/scsopt.h) for
# SelfConcordantSmoothOptimization.jl.  It adds a device-backed problem type
# whose objective and `step!` run on the MI355X; the reference's `iterate!` /
# `optim_loop!` (src/algorithms/iterate.jl) drive it unchanged.
#
# Shipped as the integration artefact; Julia is not installed in the build
# container or on the GPU box, so the executed host mirror is the Python
# package `scsopt` (same ABI, same call sequence).
module SCSOptAMD

using LinearAlgebra
using Random
using SparseArrays
using SelfConcordantSmoothOptimization
import SelfConcordantSmoothOptimization: step!, init!, ProximalMethod, ProxModel, is_interval_set

export DeviceProblem, configure!, iterate_device!, set_gram_cache!, set_solver!, rccl_unique_id, set_comm_rccl!,
       set_comm_callback!, set_test!, set_compute_f32!, fallback_counts

const lib = joinpath(@__DIR__, "..", "scsopt", "libscsopt.so")

const LOSS = Dict(:logistic_margin => 1, :logistic_ce => 2, :least_squares => 3, :quadratic => 4, :rosenbrock => 5,
                  :callback => 6)
const GGN = Dict(nothing => 0, :sigmoid_ce => 1, :linear_ls => 2)
const REG = Dict("l1" => 1, "l2" => 2, "indbox" => 3, "gl" => 4)
const SCS_ERR_REF = 5
const SCS_ERR_CALLBACK = 7

# the exception a loss callback raised on the host (the trampoline cannot throw through C):
# rethrown by chk, so a user error or the reference's MethodError reaches the caller as itself
const CB_EXCEPTION = Ref{Any}(nothing)

function chk(rc::Integer, ctx::Ptr{Cvoid})
    rc == 0 && return nothing
    if (rc == SCS_ERR_CALLBACK || rc == SCS_ERR_REF) && CB_EXCEPTION[] !== nothing
        err, CB_EXCEPTION[] = CB_EXCEPTION[], nothing
        throw(err)
    end
    msg = unsafe_string(ccall((:scs_last_error, lib), Cstring, (Ptr{Cvoid},), ctx))
    error(msg)   # SCS_ERR_REF carries the reference's own Base.error text
end

mutable struct DeviceProblem <: ProxModel
    ctx::Ptr{Cvoid}
    A
    y
    x0::Vector{Float64}
    f
    λ
    Atest
    ytest
    L
    x::Vector{Float64}
    C_set
    P
    out_fn
    grad_fx
    hess_fx
    jac_yx
    grad_fy
    hess_fy
    name
end

# devices = [d0, d1, ...]: one process drives those GPUs (scs_create_multi) -- the library splits
# the rows across them, so a plain iterate! call uses the node's GPUs with no MPI (the reference's
# iterate! is one process, iterate.jl:56-76)
# device_exchange = :host: the group's exchange through host memory instead of RCCL
# (SCS_MULTI_HOST_EXCHANGE; devices may repeat a GPU)
const SCS_MULTI_HOST_EXCHANGE = Cint(1)
function create_ctx(device::Integer, devices=nothing, device_exchange::Symbol=:rccl)
    ctx = Ref{Ptr{Cvoid}}(C_NULL)
    if devices === nothing
        rc = ccall((:scs_create, lib), Cint, (Cint, Ptr{Cvoid}, Ref{Ptr{Cvoid}}), device, C_NULL, ctx)
        rc == 0 || error("scs_create failed ($rc)")
    else
        devs = Cint.(collect(devices))
        flags = device_exchange === :host ? SCS_MULTI_HOST_EXCHANGE : Cint(0)
        rc = ccall((:scs_create_multi_ex, lib), Cint, (Ptr{Cint}, Cint, Cint, Ref{Ptr{Cvoid}}), devs, length(devs),
                   flags, ctx)
        rc == 0 || error("scs_create_multi_ex($(devs), $(device_exchange)) failed ($rc)")
    end
    return ctx[]
end

function finish_problem(ctx, A, yv, x0, loss, λ, out_fn, scale, L, sol, C_set, P)
    chk(ccall((:scs_set_loss, lib), Cint, (Ptr{Cvoid}, Cint, Cint, Float64), ctx, LOSS[loss], GGN[out_fn], scale), ctx)
    model = DeviceProblem(ctx, A, yv, x0, nothing, λ, nothing, nothing, L, sol, C_set, P, out_fn,
                          nothing, nothing, nothing, nothing, nothing, nothing)
    # optim_loop! calls model.f(model.A, model.y, x) and, with held-out data, ftest(x) =
    # model.f(model.Atest, model.ytest, x) (iterate.jl:168,173): both evaluate on the device
    model.f = (A_, y_, x) -> (A_ !== nothing && A_ === model.Atest) ? devftest(model, x) : devf(model, x)
    finalizer(m_ -> ccall((:scs_destroy, lib), Cint, (Ptr{Cvoid},), m_.ctx), model)
    return model
end

# Problem(...; Atest, ytest) (problems.jl:27-28,67-68): the held-out rows go to the device; both
# are required.  One alone is the reference's xor case (iterate.jl:170-171): the model keeps what it
# was given (so the reference's own optim_loop! takes its xor path and raises by itself at :201), and
# the device records it, so iterate_device! logs the @info and raises UndefVarError(:ftest) as well.
# Sharded: this rank's rows of Ntest_global held-out rows starting at global row test_row0.
function set_test!(model::DeviceProblem, Atest, ytest; Ntest_global::Integer=0, test_row0::Integer=0,
                   val_f32::Bool=false)
    ctx = model.ctx
    chk(ccall((:scs_set_test_data, lib), Cint,
              (Ptr{Cvoid}, Int64, Ptr{Float64}, Int64, Ptr{Float64}, Int64, Int64),
              ctx, 0, C_NULL, 0, C_NULL, 0, 0), ctx)           # clear
    model.Atest, model.ytest = nothing, nothing
    (Atest === nothing && ytest === nothing) && return model
    if xor(Atest === nothing, ytest === nothing)
        one = zeros(1)
        chk(ccall((:scs_set_test_data, lib), Cint,
                  (Ptr{Cvoid}, Int64, Ptr{Float64}, Int64, Ptr{Float64}, Int64, Int64),
                  ctx, 0, Atest === nothing ? C_NULL : pointer(one), 0, ytest === nothing ? C_NULL : pointer(one),
                  0, 0), ctx)
        model.Atest, model.ytest = Atest, ytest
        return model
    end
    yt = Vector{Float64}(vec(ytest))
    if model.grad_fx isa LossCallbacks                        # a callback loss: evaluated on the host
        model.grad_fx.test = (Atest, ytest)
        chk(ccall((:scs_set_test_callback, lib), Cint, (Ptr{Cvoid}, Cint), ctx, 1), ctx)
    elseif Atest isa SparseMatrixCSC
        At = SparseMatrixCSC(transpose(Atest))
        rowptr = Int64.(At.colptr .- 1); colidx = Int32.(At.rowval .- 1); val = Vector{Float64}(At.nzval)
        chk(ccall((:scs_set_test_sparse, lib), Cint,
                  (Ptr{Cvoid}, Int64, Int64, Ptr{Int64}, Ptr{Int32}, Ptr{Float64}, Cint, Ptr{Float64}, Int64, Int64),
                  ctx, size(Atest, 1), nnz(Atest), rowptr, colidx, val, val_f32 ? 1 : 0, yt, Ntest_global,
                  test_row0), ctx)
    else
        Am = Matrix{Float64}(Atest)
        chk(ccall((:scs_set_test_data, lib), Cint,
                  (Ptr{Cvoid}, Int64, Ptr{Float64}, Int64, Ptr{Float64}, Int64, Int64),
                  ctx, size(Am, 1), Am, size(Am, 1), yt, Ntest_global, test_row0), ctx)
    end
    model.Atest, model.ytest = Atest, ytest
    return model
end

# Problem(A, y, x0, f, λ; ...) (problems.jl:61-81) with A on the device.  Row sharding: pass
# the local rows with N_global / row0, and attach a communicator (set_comm_rccl! /
# set_comm_callback!) before the first step.
function DeviceProblem(A::Matrix{Float64}, y::AbstractVector, x0::Vector{Float64}, loss::Symbol, λ;
                       out_fn::Union{Symbol,Nothing}=nothing, scale::Float64=1.0 / size(A, 1),
                       L=nothing, sol::Vector{Float64}=zero(x0), C_set=nothing, P=nothing, device::Integer=0,
                       N_global::Integer=size(A, 1), row0::Integer=0, devices=nothing,
                       device_exchange::Symbol=:rccl, Atest=nothing,
                       ytest=nothing, Ntest_global::Integer=0, test_row0::Integer=0)
    ctx = create_ctx(device, devices, device_exchange)
    N, m = size(A)
    yv = Vector{Float64}(y)
    chk(ccall((:scs_set_data, lib), Cint,
              (Ptr{Cvoid}, Int64, Int64, Ptr{Float64}, Int64, Ptr{Float64}, Int64, Int64),
              ctx, N, m, A, N, yv, N_global, row0), ctx)
    model = finish_problem(ctx, A, yv, x0, loss, λ, out_fn, scale, L, sol, C_set, P)
    return set_test!(model, Atest, ytest; Ntest_global, test_row0)
end

# A::SparseMatrixCSC (README.md:105 builds it with sprandn): its CSC arrays are the column copy;
# the row copy is the CSC of the transpose.  0-based indices on the C side.
function DeviceProblem(A::SparseMatrixCSC{Float64}, y::AbstractVector, x0::Vector{Float64}, loss::Symbol, λ;
                       out_fn::Union{Symbol,Nothing}=nothing, scale::Float64=1.0 / size(A, 1),
                       L=nothing, sol::Vector{Float64}=zero(x0), C_set=nothing, P=nothing, device::Integer=0,
                       val_f32::Bool=false, N_global::Integer=size(A, 1), row0::Integer=0, Atest=nothing,
                       ytest=nothing, Ntest_global::Integer=0, test_row0::Integer=0)
    ctx = create_ctx(device)
    N, m = size(A)
    yv = Vector{Float64}(y)
    At = SparseMatrixCSC(transpose(A))
    rowptr = Int64.(At.colptr .- 1); colidx = Int32.(At.rowval .- 1); val = Vector{Float64}(At.nzval)
    colptr = Int64.(A.colptr .- 1);  rowidx = Int32.(A.rowval .- 1);  valT = Vector{Float64}(A.nzval)
    chk(ccall((:scs_set_sparse, lib), Cint,
              (Ptr{Cvoid}, Int64, Int64, Int64, Ptr{Int64}, Ptr{Int32}, Ptr{Float64}, Ptr{Int64}, Ptr{Int32},
               Ptr{Float64}, Cint, Ptr{Float64}, Int64, Int64),
              ctx, N, m, nnz(A), rowptr, colidx, val, colptr, rowidx, valT, val_f32 ? 1 : 0, yv, N_global, row0),
        ctx)
    model = finish_problem(ctx, A, yv, x0, loss, λ, out_fn, scale, L, sol, C_set, P)
    return set_test!(model, Atest, ytest; Ntest_global, test_row0, val_f32)
end

# ---- user losses outside the menu: the reference's own keyword callbacks ------------------
# Problem(x0, f, λ; grad_fx, hess_fx) (problems.jl:44-59) / Problem(A, y, x0, f, λ; grad_fx,
# hess_fx) (:61-81) evaluated on the host (SCS_LOSS_CALLBACK); the smoother, the solve, damping,
# prox and the loop stay on the device.  No ForwardDiff fallback: ProxLQNSCORE needs grad_fx,
# ProxNSCORE grad_fx and hess_fx.
mutable struct LossCallbacks   # mutable: `user` is pointer_from_objref(cbs), rooted by the model
    f::Function
    grad_fx::Union{Function,Nothing}
    hess_fx::Union{Function,Nothing}
    out_fn::Union{Function,Nothing}  # ProxGGNSCORE pieces (prox-GGN-SCORE.jl:44-49)
    jac_yx::Union{Function,Nothing}
    grad_fy::Union{Function,Nothing}
    hess_fy::Union{Function,Nothing}
    data::Union{Tuple,Nothing}       # (A, y) of a data problem: the closures take (A, y, x)
    nout::Int64                      # length(vec(ŷ)): the Jacobian rows (0: no GGN pieces)
    test::Union{Tuple,Nothing}       # (Atest, ytest): f(Atest, ytest, x) for SCS_CB_FTEST
end

# J, r and diag(Q) of the step: a non-diagonal Q is eigen-rotated (J̃ = VᵀJ, r̃ = Vᵀr, q = λ),
# which leaves JᵀQJ, Jᵀr and the sample-space system of ggn_score_step unchanged
function ggn_pieces!(out::Vector{Float64}, cbs::LossCallbacks, x::Vector{Float64})
    A, y = cbs.data
    n, m = cbs.nout, length(x)
    ŷ = cbs.out_fn(A, x)
    J = Matrix{Float64}(reshape(cbs.jac_yx(A, y, ŷ, x), n, m))
    r = Vector{Float64}(vec(cbs.grad_fy(A, y, ŷ)))
    Q = cbs.hess_fy(A, y, ŷ)
    if Q isa AbstractVector || isdiag(Q)
        q = Q isa AbstractVector ? Vector{Float64}(Q) : Vector{Float64}(diag(Q))
    else
        E = eigen(Symmetric(Matrix{Float64}((Q + Q') / 2)))
        J, r, q = E.vectors' * J, E.vectors' * r, E.values
    end
    out[1:n*m] .= vec(J)
    out[n*m+1:n*(m+1)] .= r
    out[n*(m+1)+1:n*(m+2)] .= q
    return nothing
end

function loss_trampoline(user::Ptr{Cvoid}, what::Cint, xp::Ptr{Float64}, m::Int64, outp::Ptr{Float64})::Cint
    cbs = unsafe_pointer_to_objref(user)::LossCallbacks
    try
        x = copy(unsafe_wrap(Array, xp, m))
        args = cbs.data === nothing ? (x,) : (cbs.data..., x)
        if what == 0
            unsafe_store!(outp, Float64(cbs.f(args...)))
        elseif what == 1
            cbs.grad_fx === nothing && error("this method needs grad_fx (no automatic differentiation on the device path)")
            copyto!(unsafe_wrap(Array, outp, m), cbs.grad_fx(args...))
        elseif what == 3
            ggn_pieces!(unsafe_wrap(Array, outp, cbs.nout * (m + 2)), cbs, x)
        elseif what == 4                                   # SCS_CB_FTEST (iterate.jl:173)
            unsafe_store!(outp, Float64(cbs.f(cbs.test..., x)))
        elseif what == 5                                   # SCS_CB_GRAD_X: ProxGGNSCORE's grad_f =
            cbs.grad_fx === nothing && error("this method needs grad_fx (no automatic differentiation on the device path)")
            if !applicable(cbs.grad_fx, x)                 # x -> model.grad_fx(x) (prox-GGN-SCORE.jl:58-59)
                CB_EXCEPTION[] = MethodError(cbs.grad_fx, (x,))
                return Cint(2)                             # SCS_CB_NO_METHOD -> SCS_ERR_REF
            end
            copyto!(unsafe_wrap(Array, outp, m), cbs.grad_fx(x))
        else
            cbs.hess_fx === nothing && error("ProxNSCORE needs hess_fx (no automatic differentiation on the device path)")
            copyto!(unsafe_wrap(Array, outp, m * m), vec(Matrix{Float64}(cbs.hess_fx(args...))))   # column-major
        end
        return Cint(0)
    catch err
        CB_EXCEPTION[] = err
        return Cint(1)
    end
end

function callback_problem(cbs::LossCallbacks, x0::Vector{Float64}, λ, L, sol, C_set, P, device)
    ctx = create_ctx(device)
    m = length(x0)
    chk(ccall((:scs_set_data, lib), Cint,
              (Ptr{Cvoid}, Int64, Int64, Ptr{Float64}, Int64, Ptr{Float64}, Int64, Int64),
              ctx, 0, m, C_NULL, 0, C_NULL, 0, 0), ctx)
    model = finish_problem(ctx, nothing, nothing, x0, :callback, λ, nothing, 1.0, L, sol, C_set, P)
    model.grad_fx = cbs                         # rooted with the model: `user` points at it
    fp = @cfunction(loss_trampoline, Cint, (Ptr{Cvoid}, Cint, Ptr{Float64}, Int64, Ptr{Float64}))
    chk(ccall((:scs_set_loss_callback, lib), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Cvoid}, Int64),
              ctx, fp, pointer_from_objref(cbs), cbs.nout), ctx)
    return model
end

DeviceProblem(x0::Vector{Float64}, f::Function, λ; grad_fx=nothing, hess_fx=nothing, L=nothing,
              sol::Vector{Float64}=zero(x0), C_set=nothing, P=nothing, device::Integer=0) =
    callback_problem(LossCallbacks(f, grad_fx, hess_fx, nothing, nothing, nothing, nothing, nothing, 0, nothing),
                     x0, λ, L, sol, C_set, P, device)

# y may be a matrix (ny > 1 outputs, iterate.jl:105-107): out_fn / jac_yx / grad_fy / hess_fy see it as is
function DeviceProblem(A::AbstractMatrix, y::AbstractVecOrMat, x0::Vector{Float64}, f::Function, λ; grad_fx=nothing,
                       hess_fx=nothing, out_fn=nothing, jac_yx=nothing, grad_fy=nothing, hess_fy=nothing,
                       L=nothing, sol::Vector{Float64}=zero(x0), C_set=nothing, P=nothing, device::Integer=0,
                       Atest=nothing, ytest=nothing)
    ggn = all(!isnothing, (out_fn, jac_yx, grad_fy, hess_fy))
    nout = ggn ? Int64(length(out_fn(A, x0))) : 0
    cbs = LossCallbacks(f, grad_fx, hess_fx, out_fn, jac_yx, grad_fy, hess_fy, (A, y), nout, nothing)
    model = callback_problem(cbs, x0, λ, L, sol, C_set, P, device)
    return set_test!(model, Atest, ytest)
end

# ---- row sharding (SURVEY.md §8e): one process per GPU, A's rows split across them ---------
# libscsopt's own RCCL communicator: rank 0 draws the id, the caller hands the 128 bytes to
# every rank (MPI.jl's Bcast!, a shared file ...), every rank then calls set_comm_rccl!.
function rccl_unique_id()
    id = zeros(UInt8, 128)
    rc = ccall((:scs_rccl_unique_id, lib), Cint, (Ptr{Cvoid},), id)
    rc == 0 || error("scs_rccl_unique_id failed ($rc)")
    return id
end

function set_comm_rccl!(model::DeviceProblem, rank::Integer, nranks::Integer, id::Vector{UInt8})
    length(id) == 128 || error("an RCCL unique id is 128 bytes")
    chk(ccall((:scs_set_comm_rccl, lib), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{Cvoid}), model.ctx, rank, nranks, id),
        model.ctx)
    return model
end

# Or any all-reduce the host owns: `sum!(buf::Ptr{Float64}, count::Int64, stream::Ptr{Cvoid})`
# sums `count` doubles in place across ranks on the device (e.g. an RCCL call through
# AMDGPU.jl); the payload lives in a device buffer of reduce_buffer_size doubles registered here.
const CALLBACKS = Dict{Ptr{Cvoid},Any}()

function allreduce_trampoline(buf::Ptr{Cvoid}, count::Int64, stream::Ptr{Cvoid}, user::Ptr{Cvoid})::Cint
    try
        CALLBACKS[user](Ptr{Float64}(buf), count, stream)
        return Cint(0)
    catch
        return Cint(1)
    end
end

function set_comm_callback!(model::DeviceProblem, rank::Integer, nranks::Integer, sum!::Function,
                            dev_buf::Ptr{Cvoid}=C_NULL)
    CALLBACKS[model.ctx] = sum!
    fn = @cfunction(allreduce_trampoline, Cint, (Ptr{Cvoid}, Int64, Ptr{Cvoid}, Ptr{Cvoid}))
    chk(ccall((:scs_set_comm, lib), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{Cvoid}, Ptr{Cvoid}),
              model.ctx, rank, nranks, fn, model.ctx), model.ctx)
    if dev_buf != C_NULL
        n = Ref{Int64}(0)
        chk(ccall((:scs_reduce_buffer_size, lib), Cint, (Ptr{Cvoid}, Ref{Int64}), model.ctx, n), model.ctx)
        chk(ccall((:scs_set_reduce_buffer, lib), Cint, (Ptr{Cvoid}, Ptr{Cvoid}, Int64), model.ctx, dev_buf, n[]),
            model.ctx)
    end
    return model
end

function devf(model::DeviceProblem, x::Vector{Float64})
    out = Ref{Float64}(0.0)
    chk(ccall((:scs_eval_f, lib), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ref{Float64}), model.ctx, x, out), model.ctx)
    return out[]
end

function devftest(model::DeviceProblem, x::Vector{Float64})
    out = Ref{Float64}(0.0)
    chk(ccall((:scs_eval_ftest, lib), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ref{Float64}), model.ctx, x, out), model.ctx)
    return out[]
end

"""configure!(model, reg_name, hμ): push reg_name/λ/C_set/P and the smoother to the device."""
function configure!(model::DeviceProblem, reg_name::String, hμ)
    haskey(REG, reg_name) || error("reg_name not valid.")
    lam = Float64.(collect(model.λ isa Number ? (model.λ,) : model.λ))
    lb = ub = Float64[]; nb = 0
    ind = Int64[]; ng = 0
    if reg_name == "indbox"
        lb, ub = cset_bounds(model.C_set); nb = length(lb)
    elseif reg_name == "gl"
        ind = Int64.(vec(model.P.ind)); ng = size(model.P.ind, 2)     # column-major 3 x G, 1-based
    end
    chk(ccall((:scs_set_reg, lib), Cint,
              (Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Ptr{Float64}, Ptr{Float64}, Int64, Ptr{Int64}, Int64),
              model.ctx, REG[reg_name], lam, length(lam), lb, ub, nb, ind, ng), model.ctx)
    if reg_name == "gl"                                  # P.matrix*x = x[G] in get_reg
        G = Int64.(model.P.G)
        chk(ccall((:scs_set_group_map, lib), Cint, (Ptr{Cvoid}, Ptr{Int64}, Int64), model.ctx, G, length(G)),
            model.ctx)
    end
    kind, slb, sub = smoother_kind(hμ, model)
    chk(ccall((:scs_set_smoother, lib), Cint,
              (Ptr{Cvoid}, Cint, Float64, Float64, Float64, Ptr{Float64}, Ptr{Float64}, Int64),
              model.ctx, kind, hμ.μ, hμ.Mh, hμ.ν, slb, sub, length(slb)), model.ctx)
    chk(ccall((:scs_set_L, lib), Cint, (Ptr{Cvoid}, Cint, Float64), model.ctx, model.L === nothing ? 0 : 1,
              model.L === nothing ? 0.0 : Float64(model.L)), model.ctx)
    return model
end

# C_set -> (lb, ub) exactly as prox_step(::scaled_proximal_indbox) reads it
# (prox-operators.jl:34-46): an interval, a tuple of intervals, or a (lb, ub) pair / vector.
function cset_bounds(C_set)
    C_set === nothing && error("indbox needs model.C_set")
    if is_interval_set(C_set)
        lb, ub = C_set isa Tuple ? ([minimum.(C_set)...], [maximum.(C_set)...]) : (minimum(C_set), maximum(C_set))
    else
        lb, ub = C_set[1], C_set[2]
    end
    return Float64.(vcat(lb)), Float64.(vcat(ub))
end

# The IndBox smoothers keep their bounds only in the closures they build
# (phuber-smooth.jl:59-65, exponential-smooth.jl:28-34, log-exp-smooth.jl:28-34:
# `grad = (Cmat,x) -> huber_grad_indbox(x; μ=mu, lb=lb, ub=ub)`), so the captured `lb` / `ub`
# are read off the closure object (a closure's captures are its fields); model.C_set is the
# fallback for a hand-built smoother whose closure captured other names.
function indbox_bounds(hμ, model)
    g = hμ.grad
    if hasfield(typeof(g), :lb) && hasfield(typeof(g), :ub)
        return Float64.(vcat(getfield(g, :lb))), Float64.(vcat(getfield(g, :ub)))
    end
    return cset_bounds(model.C_set)
end

# smoother struct -> (kind, lb, ub)
function smoother_kind(hμ, model)
    T = typeof(hμ)
    T <: PHuberSmootherL1L2 && return (1, Float64[], Float64[])
    T <: PHuberSmootherIndBox && return (2, indbox_bounds(hμ, model)...)
    T <: PHuberSmootherGL && return (3, Float64[], Float64[])
    T <: ExponentialSmootherIndBox && return (4, indbox_bounds(hμ, model)...)
    T <: LogExpSmootherIndBox && return (5, indbox_bounds(hμ, model)...)
    T <: OsBaSmootherL1L2 && return (6, Float64[], Float64[])
    T <: OsBaSmootherGL && return (7, Float64[], Float64[])
    error("smoother $(T) has no device implementation")
end

# Opt-in reuse of the x-independent AᵀQA of least squares across steps (scs_set_gram_cache);
# the reference recomputes it every step (prox-GGN-SCORE.jl:129) and that stays the default.
set_gram_cache!(model::DeviceProblem, on::Bool=true) =
    chk(ccall((:scs_set_gram_cache, lib), Cint, (Ptr{Cvoid}, Cint), model.ctx, on ? 1 : 0), model.ctx)

# The reference's own factorizations (scs_set_solver): Householder QR for ProxGGNSCORE's systems
# (prox-GGN-SCORE.jl:126,131), LU for ProxNSCORE's -- the default is Cholesky with the LU fallback.
set_solver!(model::DeviceProblem, reference::Bool=true) =
    chk(ccall((:scs_set_solver, lib), Cint, (Ptr{Cvoid}, Cint), model.ctx, reference ? 1 : 0), model.ctx)

# The compute arm of the fp32-vs-fp64 study (BASELINE configs[4]): fp32 arithmetic in the sparse
# products of fp32-stored values (val_f32 = true) and the L-BFGS two-loop (scs_set_compute_f32).
set_compute_f32!(model::DeviceProblem, on::Bool=true) =
    chk(ccall((:scs_set_compute_f32, lib), Cint, (Ptr{Cvoid}, Cint), model.ctx, on ? 1 : 0), model.ctx)

# The fallbacks taken instead of failing since the problem's context was created (scs_fallback_counts;
# SCS_FB_* in include/scsopt.h, in that order), as name => count.
const FALLBACKS = (:lu_coop_refused, :lu_coop_redo, :solve_blocks, :qr_blocks, :chain_redo, :pipe_redo,
                   :qr_coop_refused, :qr_coop_redo)
function fallback_counts(model::DeviceProblem)
    out = zeros(Int64, length(FALLBACKS))
    chk(ccall((:scs_fallback_counts, lib), Cint, (Ptr{Cvoid}, Ptr{Int64}, Cint), model.ctx, out, length(out)),
        model.ctx)
    return Dict(zip(FALLBACKS, out))
end

method_code(m) = m isa ProxNSCORE ? 1 : m isa ProxGGNSCORE ? 2 : m isa ProxLQNSCORE ? 3 : error("unknown method")

# init!(method, x) for device problems (prox-L-BFGS-SCORE.jl:31-36)
function init_device!(method::ProximalMethod, model::DeviceProblem)
    mem = method isa ProxLQNSCORE ? method.m : 0
    chk(ccall((:scs_method_init, lib), Cint, (Ptr{Cvoid}, Cint, Cint, Cint, Cint),
              model.ctx, method_code(method), method.ss_type, method.use_prox, mem), model.ctx)
end

# step! on a DeviceProblem: the whole per-iteration work runs in libscsopt.
function step!(method::ProximalMethod, model::DeviceProblem, reg_name, hμ, As, x, x_prev, ys, Cmat, iter;
               ∇fx=nothing, return_dx=false)
    # the device holds the rows: a minibatch As from the reference's loader cannot be mapped back
    # to them, so minibatches go through iterate_device!(...; batch_size) (scs_set_batches)
    As === nothing || size(As, 1) == size(model.A, 1) ||
        error("minibatch As on a DeviceProblem: use iterate_device!(...; batch_size, shuffle_batch)")
    x_new = similar(x); dx = similar(x); pri = Ref{Float64}(0.0)
    # ∇fx (iterate.jl:52-54): grad_f = x -> ∇fx inside the step (prox-L-BFGS-SCORE.jl:98-100)
    g = ∇fx === nothing ? C_NULL : Vector{Float64}(vec(∇fx))
    g === C_NULL || length(g) == length(x) || error("∇fx must have length(x) entries")
    chk(ccall((:scs_step_grad, lib), Cint,
              (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Int64, Ptr{Float64}, Ptr{Float64}, Ptr{Float64}, Ref{Float64}),
              model.ctx, x, x_prev, iter, g, x_new, dx, pri), model.ctx)
    return return_dx ? (x_new, dx, pri[]) : (x_new, pri[])
end

# The collected loader batches of optim_loop! (iterate.jl:124-146, utils.jl:14-25) as 0-based
# row lists: ceil(N/b) consecutive runs of the (randperm-shuffled) sample order, the last one
# partial; slice_samples keeps only sample 1 (max_iter stays 1); local_max_iter truncates.
# `nothing` = the one full batch.
function loader_batches(N::Int, batch_size, slice_samples::Bool, shuffle_batch::Bool, local_max_iter)
    batch_size !== nothing && slice_samples && (slice_samples = false)
    max_iter = batch_size !== nothing ? Int(ceil(N / batch_size)) : 1
    iend = (local_max_iter !== nothing && Int(floor(local_max_iter)) > 0) ?
           min(Int(floor(local_max_iter)), max_iter) : max_iter
    slice_samples && return [Int64[i - 1] for i in 1:min(iend, N)]
    batch_size === nothing && return nothing
    order = shuffle_batch ? randperm(N) .- 1 : collect(0:N-1)
    return [Int64.(order[(i-1)*batch_size+1:min(i * batch_size, N)]) for i in 1:iend]
end

function set_batches!(model::DeviceProblem, batches)
    if batches === nothing || isempty(batches)
        chk(ccall((:scs_set_batches, lib), Cint, (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int64}, Int64),
                  model.ctx, C_NULL, C_NULL, 0), model.ctx)
        return
    end
    rows = reduce(vcat, batches)
    offs = Int64[0; cumsum(length.(batches))]
    chk(ccall((:scs_set_batches, lib), Cint, (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int64}, Int64),
              model.ctx, rows, offs, length(batches)), model.ctx)
end

# iterate!(method, model::DeviceProblem, reg_name, hμ; max_epoch, x_tol, f_tol, batch_size, ...):
# optim_loop! (iterate.jl:100-267) as ONE ccall (scs_iterate) -- no per-epoch host round trips;
# minibatches are gathered on the device from the registered row lists (scs_set_batches).
# Returns the reference's Solution (iterate.jl:3-32); pri_res_norm[1] is `nothing` as there.
# The rows of all ranks (scs_get_dims): the loader's N on a row-sharded problem.
function global_rows(model::DeviceProblem)
    Ng = Ref{Int64}(0)
    chk(ccall((:scs_get_dims, lib), Cint, (Ptr{Cvoid}, Ptr{Int64}, Ptr{Int64}, Ref{Int64}, Ptr{Int64}),
              model.ctx, C_NULL, C_NULL, Ng, C_NULL), model.ctx)
    Ng[]
end

# Row-sharded minibatches: every rank registers the same GLOBAL batch list and keeps its own rows
# of each batch; `bcast` (e.g. `b -> MPI.bcast(b, 0, comm)`) hands rank 0's shuffled list to all.
function iterate_device!(method::ProximalMethod, model::DeviceProblem, reg_name::String, hμ;
                         α=nothing, batch_size=nothing, slice_samples=false, shuffle_batch=true,
                         max_epoch=1000, local_max_iter=nothing, x_tol=1e-10, f_tol=1e-10, bcast=identity)
    local_max_iter === nothing || (max_epoch = 1)      # iterate.jl:66
    α === nothing || (model.L = 1 / α)                 # iterate.jl:113-115
    batches = (batch_size !== nothing || slice_samples) ?
              bcast(loader_batches(Int(global_rows(model)), batch_size, slice_samples, shuffle_batch,
                                   local_max_iter)) : nothing
    set_batches!(model, batches)
    try
        return iterate_registered!(method, model, reg_name, hμ, max_epoch, x_tol, f_tol)
    finally
        batches === nothing || set_batches!(model, nothing)
    end
end

function iterate_registered!(method, model, reg_name, hμ, max_epoch, x_tol, f_tol)
    configure!(model, reg_name, hμ)
    init_device!(method, model)
    cap = 2 * max_epoch + 1                           # scsopt.h: up to two pushes per epoch
    obj, fval, pri, rel, objrel, tms, ftst = (Vector{Float64}(undef, cap) for _ in 1:7)
    has_test = model.Atest !== nothing && model.ytest !== nothing   # iterate.jl:169-175: Solution.fvaltest
    xor_test = xor(model.Atest === nothing, model.ytest === nothing)
    xor_test && @info "Both input (Atest) and target (ytest) data are required for testing the model, but only one of these has been provided.\nWill skip testing..."
    hist = (pointer(obj), pointer(fval), pointer(pri), pointer(rel), pointer(objrel), pointer(tms),
            has_test ? pointer(ftst) : Ptr{Float64}(C_NULL))
    x_out = similar(model.x0); nh = Ref{Int64}(0); ep = Ref{Int64}(0)
    GC.@preserve obj fval pri rel objrel tms ftst begin
        rc = ccall((:scs_iterate_ex, lib), Cint,
                   (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Int64, Float64, Float64, Cint, Ptr{Float64},
                    Ref{NTuple{7,Ptr{Float64}}}, Csize_t, Ref{Int64}, Ref{Int64}),
                   model.ctx, model.x0, model.x, max_epoch, x_tol, f_tol, reg_name == "gl" ? 1 : 0, x_out,
                   hist, sizeof(NTuple{7,Ptr{Float64}}), nh, ep)
        # the xor case fails at the first stats push, as show_stat! does at iterate.jl:201
        (xor_test && rc == SCS_ERR_REF) && throw(UndefVarError(:ftest))
        chk(rc, model.ctx)
    end
    n = nh[]
    pris = Any[isnan(pri[i]) && i == 1 ? nothing : pri[i] for i in 1:n]
    return Solution(x_out, obj[1:n], fval[1:n], pris, has_test ? ftst[1:n] : [], rel[1:n], objrel[1:n], Dict(),
                    tms[1:n], ep[], model)
end

end # module
