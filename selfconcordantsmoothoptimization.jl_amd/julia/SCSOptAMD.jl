# SCSOptAMD.jl -- Julia `ccall` binding of libscsopt (include/scsopt.h) for
# SelfConcordantSmoothOptimization.jl.  It adds a device-backed problem type
# whose objective and `step!` run on the MI355X; the reference's `iterate!` /
# `optim_loop!` (src/algorithms/iterate.jl) drive it unchanged.
#
# Shipped as the integration artefact; Julia is not installed in the build
# container or on the GPU box, so the executed host mirror is the Python
# package `scsopt` (same ABI, same call sequence).
module SCSOptAMD

using SelfConcordantSmoothOptimization
import SelfConcordantSmoothOptimization: step!, init!, ProximalMethod, ProxModel

export DeviceProblem, configure!

const lib = joinpath(@__DIR__, "..", "scsopt", "libscsopt.so")

const LOSS = Dict(:logistic_margin => 1, :logistic_ce => 2, :least_squares => 3, :quadratic => 4, :rosenbrock => 5)
const GGN = Dict(nothing => 0, :sigmoid_ce => 1, :linear_ls => 2)
const REG = Dict("l1" => 1, "l2" => 2, "indbox" => 3, "gl" => 4)
const SCS_ERR_REF = 5

function chk(rc::Integer, ctx::Ptr{Cvoid})
    rc == 0 && return nothing
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

function DeviceProblem(A::Matrix{Float64}, y::AbstractVector, x0::Vector{Float64}, loss::Symbol, λ;
                       out_fn::Union{Symbol,Nothing}=nothing, scale::Float64=1.0 / size(A, 1),
                       L=nothing, sol::Vector{Float64}=zero(x0), C_set=nothing, P=nothing, device::Integer=0)
    ctx = Ref{Ptr{Cvoid}}(C_NULL)
    rc = ccall((:scs_create, lib), Cint, (Cint, Ptr{Cvoid}, Ref{Ptr{Cvoid}}), device, C_NULL, ctx)
    rc == 0 || error("scs_create failed ($rc)")
    N, m = size(A)
    yv = Vector{Float64}(y)
    chk(ccall((:scs_set_data, lib), Cint,
              (Ptr{Cvoid}, Int64, Int64, Ptr{Float64}, Int64, Ptr{Float64}, Int64, Int64),
              ctx[], N, m, A, N, yv, N, 0), ctx[])
    chk(ccall((:scs_set_loss, lib), Cint, (Ptr{Cvoid}, Cint, Cint, Float64), ctx[], LOSS[loss], GGN[out_fn], scale),
        ctx[])
    model = DeviceProblem(ctx[], A, yv, x0, nothing, λ, nothing, nothing, L, sol, C_set, P, out_fn,
                          nothing, nothing, nothing, nothing, nothing, nothing)
    model.f = (A_, y_, x) -> devf(model, x)        # optim_loop! calls model.f(model.A, model.y, x)
    finalizer(m_ -> ccall((:scs_destroy, lib), Cint, (Ptr{Cvoid},), m_.ctx), model)
    return model
end

function devf(model::DeviceProblem, x::Vector{Float64})
    out = Ref{Float64}(0.0)
    chk(ccall((:scs_eval_f, lib), Cint, (Ptr{Cvoid}, Ptr{Float64}, Ref{Float64}), model.ctx, x, out), model.ctx)
    return out[]
end

"""configure!(model, reg_name, hμ): push reg_name/λ/C_set/P and the smoother to the device."""
function configure!(model::DeviceProblem, reg_name::String, hμ)
    haskey(REG, reg_name) || error("reg_name not valid.")
    lam = Float64.(collect(model.λ isa Number ? (model.λ,) : model.λ))
    lb = ub = Float64[]; nb = 0
    ind = Int64[]; ng = 0
    if reg_name == "indbox"
        lb = Float64.(vcat(model.C_set[1])); ub = Float64.(vcat(model.C_set[2])); nb = length(lb)
    elseif reg_name == "gl"
        ind = Int64.(vec(model.P.ind)); ng = size(model.P.ind, 2)     # column-major 3 x G, 1-based
    end
    chk(ccall((:scs_set_reg, lib), Cint,
              (Ptr{Cvoid}, Cint, Ptr{Float64}, Cint, Ptr{Float64}, Ptr{Float64}, Int64, Ptr{Int64}, Int64),
              model.ctx, REG[reg_name], lam, length(lam), lb, ub, nb, ind, ng), model.ctx)
    kind, slb, sub = smoother_kind(hμ)
    chk(ccall((:scs_set_smoother, lib), Cint,
              (Ptr{Cvoid}, Cint, Float64, Float64, Float64, Ptr{Float64}, Ptr{Float64}, Int64),
              model.ctx, kind, hμ.μ, hμ.Mh, hμ.ν, slb, sub, length(slb)), model.ctx)
    chk(ccall((:scs_set_L, lib), Cint, (Ptr{Cvoid}, Cint, Float64), model.ctx, model.L === nothing ? 0 : 1,
              model.L === nothing ? 0.0 : Float64(model.L)), model.ctx)
    return model
end

# smoother struct -> (kind, lb, ub); the IndBox smoothers' bounds live in their closures,
# so callers pass them through `hμ.lb/hμ.ub` when wrapping (PHuberSmootherIndBox(lb, ub, μ)).
function smoother_kind(hμ)
    T = typeof(hμ)
    T <: PHuberSmootherL1L2 && return (1, Float64[], Float64[])
    T <: PHuberSmootherIndBox && return (2, Float64.(vcat(hμ.lb)), Float64.(vcat(hμ.ub)))
    T <: PHuberSmootherGL && return (3, Float64[], Float64[])
    T <: ExponentialSmootherIndBox && return (4, Float64.(vcat(hμ.lb)), Float64.(vcat(hμ.ub)))
    T <: LogExpSmootherIndBox && return (5, Float64.(vcat(hμ.lb)), Float64.(vcat(hμ.ub)))
    T <: OsBaSmootherL1L2 && return (6, Float64[], Float64[])
    T <: OsBaSmootherGL && return (7, Float64[], Float64[])
    error("smoother $(T) has no device implementation")
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
    x_new = similar(x); dx = similar(x); pri = Ref{Float64}(0.0)
    chk(ccall((:scs_step, lib), Cint,
              (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Int64, Ptr{Float64}, Ptr{Float64}, Ref{Float64}),
              model.ctx, x, x_prev, iter, x_new, dx, pri), model.ctx)
    return return_dx ? (x_new, dx, pri[]) : (x_new, pri[])
end

# iterate!(method, model::DeviceProblem, reg_name, hμ; max_epoch, x_tol, f_tol): optim_loop!
# (iterate.jl:100-267) as ONE ccall (scs_iterate) -- no per-epoch host round trips.  Returns the
# reference's Solution (iterate.jl:3-32); pri_res_norm[1] is `nothing` as in the reference.
function iterate_device!(method::ProximalMethod, model::DeviceProblem, reg_name::String, hμ;
                         α=nothing, max_epoch=1000, x_tol=1e-10, f_tol=1e-10)
    α === nothing || (model.L = 1 / α)                 # iterate.jl:113-115
    configure!(model, reg_name, hμ)
    init_device!(method, model)
    cap = max_epoch + 1
    obj, fval, pri, rel, objrel, tms = (Vector{Float64}(undef, cap) for _ in 1:6)
    hist = (pointer(obj), pointer(fval), pointer(pri), pointer(rel), pointer(objrel), pointer(tms))
    x_out = similar(model.x0); nh = Ref{Int64}(0); ep = Ref{Int64}(0)
    GC.@preserve obj fval pri rel objrel tms begin
        chk(ccall((:scs_iterate, lib), Cint,
                  (Ptr{Cvoid}, Ptr{Float64}, Ptr{Float64}, Int64, Float64, Float64, Cint, Ptr{Float64},
                   Ref{NTuple{6,Ptr{Float64}}}, Ref{Int64}, Ref{Int64}),
                  model.ctx, model.x0, model.x, max_epoch, x_tol, f_tol, reg_name == "gl" ? 1 : 0, x_out,
                  hist, nh, ep), model.ctx)
    end
    n = nh[]
    pris = Any[isnan(pri[i]) && i == 1 ? nothing : pri[i] for i in 1:n]
    return Solution(x_out, obj[1:n], fval[1:n], pris, [], rel[1:n], objrel[1:n], Dict(), tms[1:n], ep[], model)
end

end # module
