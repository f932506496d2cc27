"""
    TensorKrylovHIP

Drop-in MI355X backend for TensorKrylov.jl's inner Krylov iteration.  Adds three
orthonormalization types,

    HIPTensorArnoldi, HIPTensorLanczos, HIPTensorLanczosReorth  <: TensorDecomposition

whose per-factor steps (SpMV + MGS / TTR, update_rhs!'s dots, the orthogonality Gram
rows) and basis_tensor_mul! run in libtkhip.so (include/tk.h) on a gfx950 GPU, so that

    solve_tensorized_system(system, nmax, HIPTensorLanczosReorth, tol)

works unchanged.  The host keeps only what tensorkrylov! reads on the host (src/
tensor_krylov_method.jl:36-125): H_s (k x k minors and H_s[k+1,k]) and btilde_s; V_s
stays on the device and is exposed as `HIPBasis <: AbstractMatrix{Float64}`, which
answers dot (update_rhs!, src/utils.jl:466-476), basis_tensor_mul! (src/utils.jl:478-488)
and orthogonality_loss (src/orthogonal_bases.jl:231-257) from the step records or by one
library call.

Not exercised in the build container (no Julia there); see INTEGRATION.md.
"""
module TensorKrylovHIP

using LinearAlgebra, SparseArrays
using TensorKrylov
import TensorKrylov: orthonormalize!, tensorkrylov!, orthogonality_loss
using TensorKrylov: KronComp, KronMat, KronProd, Instance, KruskalTensor, ConvergenceData,
                    TensorDecomposition, Arnoldi, Lanczos, LanczosReorth
import LinearAlgebra: mul!, dot

export HIPTensorArnoldi, HIPTensorLanczos, HIPTensorLanczosReorth, HIPBasis, libtkhip

const libtkhip = get(ENV, "TKHIP_LIB", joinpath(@__DIR__, "..", "tkamd", "libtkhip.so"))

const TK_ARNOLDI, TK_LANCZOS, TK_LANCZOS_REORTH = Cint(0), Cint(1), Cint(2)

tk_error() = unsafe_string(ccall((:tk_last_error, libtkhip), Cstring, ()))
check(st::Cint) = st == 0 || error("libtkhip: " * tk_error())

# ------------------------------------------------------------------ context / matrices
mutable struct HIPContext
    h::Ptr{Cvoid}
    function HIPContext(device::Integer = 0)
        r = Ref{Ptr{Cvoid}}(C_NULL)
        check(ccall((:tk_ctx_create, libtkhip), Cint, (Cint, Ref{Ptr{Cvoid}}), device, r))
        c = new(r[])
        finalizer(x -> ccall((:tk_ctx_destroy, libtkhip), Cint, (Ptr{Cvoid},), x.h), c)
    end
end

const DEFAULT_CTX = Ref{Union{Nothing, HIPContext}}(nothing)
context() = something(DEFAULT_CTX[], (DEFAULT_CTX[] = HIPContext(0)))

mutable struct HIPMatrix
    h::Ptr{Cvoid}
    n::Int
    ctx::HIPContext
    # SparseMatrixCSC{Float64,Int64} fields go over unchanged (1-based)
    function HIPMatrix(ctx::HIPContext, A::SparseMatrixCSC{Float64, Int64})
        r = Ref{Ptr{Cvoid}}(C_NULL)
        check(ccall((:tk_matrix_from_csc, libtkhip), Cint,
                    (Ptr{Cvoid}, Int64, Ptr{Int64}, Ptr{Int64}, Ptr{Float64}, Cint, Ref{Ptr{Cvoid}}),
                    ctx.h, size(A, 1), A.colptr, A.rowval, A.nzval, 1, r))
        m = new(r[], size(A, 1), ctx)
        finalizer(x -> ccall((:tk_matrix_destroy, libtkhip), Cint, (Ptr{Cvoid},), x.h), m)
    end
end
HIPMatrix(ctx::HIPContext, A::AbstractMatrix) = HIPMatrix(ctx, SparseMatrixCSC{Float64, Int64}(sparse(A)))

# ------------------------------------------------------------------ device decomposition
reclen(kmax) = 2kmax + 10

mutable struct HIPDecomp
    h::Ptr{Cvoid}
    d::Int
    n::Int
    kmax::Int
    m::Int
    mats::Vector{HIPMatrix}
    b::Vector{Vector{Float64}}
end

function HIPDecomp(ctx::HIPContext, method::Cint, mats::Vector{HIPMatrix}, b, kmax::Int)
    d = length(mats)
    bs = [Vector{Float64}(x) for x in b]
    r = Ref{Ptr{Cvoid}}(C_NULL)
    check(ccall((:tk_decomp_create, libtkhip), Cint,
                (Ptr{Cvoid}, Cint, Cint, Cint, Cint, Ptr{Ptr{Cvoid}}, Ptr{Ptr{Float64}}, Int64, Cint, Cint,
                 Ref{Ptr{Cvoid}}),
                ctx.h, method, d, 0, d, [m.h for m in mats], [pointer(x) for x in bs], mats[1].n, kmax,
                2 #= factor 1's Gram rows per step: orthogonality_loss is read every iteration =#, r))
    dc = HIPDecomp(r[], d, mats[1].n, kmax, reclen(kmax), mats, bs)
    finalizer(x -> ccall((:tk_decomp_destroy, libtkhip), Cint, (Ptr{Cvoid},), x.h), dc)
end

# the record of one call: column-major m x d (C's [d][m])
function records(dc::HIPDecomp, f::Symbol, args...)
    rec = zeros(dc.m, dc.d)
    if f === :init
        check(ccall((:tk_decomp_init, libtkhip), Cint, (Ptr{Cvoid}, Ptr{Float64}), dc.h, rec))
    else
        check(ccall((:tk_decomp_step, libtkhip), Cint, (Ptr{Cvoid}, Cint, Ptr{Float64}), dc.h, args[1], rec))
    end
    return rec
end

# ------------------------------------------------------------------ device-backed basis
"""
    HIPBasis

The leading `ncols` columns of V_s of one factor, resident on the GPU.  tensorkrylov!
only touches V through `principal_minors(V, n, k)`, `kth_columns(V, k)`,
`dot(V_s[:, k], b_s)`, `basis_tensor_mul!` and `orthogonality_loss`; each is answered
from the step records or by one library call.  Plain getindex copies a column to the host.
"""
struct HIPBasis <: AbstractMatrix{Float64}
    dc::HIPDecomp
    s::Int                               # factor index (1-based)
    ncols::Int                           # V_s[:, 1:ncols]
    btilde::Vector{Float64}              # <V[:,c], b_s> from the records (shared by all prefixes)
    gram::Matrix{Float64}                # Gram rows (factor 1 / LanczosReorth)
end
HIPBasis(V::HIPBasis, k::Int) = HIPBasis(V.dc, V.s, k, V.btilde, V.gram)
Base.size(V::HIPBasis) = (V.dc.n, V.ncols)
function column(V::HIPBasis, c::Int)
    out = zeros(V.dc.n)
    check(ccall((:tk_decomp_get_basis, libtkhip), Cint, (Ptr{Cvoid}, Cint, Cint, Cint, Ptr{Float64}),
                V.dc.h, V.s - 1, c - 1, 1, out))
    return out
end
Base.getindex(V::HIPBasis, i::Int, j::Int) = column(V, j)[i]

# principal_minors(V, n, k) (src/tensor_struct.jl:398-402): prefixes instead of SubArrays, so
# the result is again a KronComp{HIPBasis} without copying V to the host
TensorKrylov.principal_minors(V::KronComp{HIPBasis}, i::Int, j::Int) =
    (i == first(V.M).dc.n || error("row minors of a device basis are not supported");
     KronComp{HIPBasis}([HIPBasis(Vs, j) for Vs in V.M]))

const HIPCol = SubArray{Float64, 1, HIPBasis, <:Tuple{Base.Slice, Int}}

# update_rhs! (src/utils.jl:472): dot(V[s][:, k], b[s]) was computed by the step kernels
function dot(x::HIPCol, b::AbstractVector{Float64})
    V = parent(x)
    k = parentindices(x)[2]
    b === V.dc.b[V.s] || b == V.dc.b[V.s] ? V.btilde[k] : dot(column(V, k), b)
end

# basis_tensor_mul! (src/utils.jl:478-488): X_s = V_s[:, 1:k] * Y_s for all factors, one MFMA launch
function TensorKrylov.basis_tensor_mul!(x::KruskalTensor{Float64}, V::KronComp{HIPBasis},
                                        y::KruskalTensor{Float64})
    x.lambda = copy(y.lambda)
    dc = first(V.M).dc
    k = first(V.M).ncols
    t = size(y.fmat[1], 2)
    Ys = zeros(k, t, dc.d)
    for s in 1:dc.d
        Ys[:, :, s] .= y.fmat[s]
    end
    Xs = zeros(dc.n, t, dc.d)
    check(ccall((:tk_decomp_basis_mul, libtkhip), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{Float64}, Ptr{Float64}),
                dc.h, k, t, Ys, Xs))
    for s in 1:dc.d
        x.fmat[s] .= @view Xs[:, :, s]
    end
    return x
end

# single-factor mul! (same kernel; other factors get Y = 0)
function mul!(X::Matrix{Float64}, V::HIPBasis, Y::Matrix{Float64})
    k, t = V.ncols, size(Y, 2)
    Ys = zeros(k, t, V.dc.d)
    Ys[:, :, V.s] .= Y
    Xs = zeros(V.dc.n, t, V.dc.d)
    check(ccall((:tk_decomp_basis_mul, libtkhip), Cint, (Ptr{Cvoid}, Cint, Cint, Ptr{Float64}, Ptr{Float64}),
                V.dc.h, k, t, Ys, Xs))
    X .= @view Xs[:, :, V.s]
    return X
end

# orthogonality_loss(V, k) = norm(V[:,1:k]'V[:,1:k] - I) (src/orthogonal_bases.jl:250-257)
# from the Gram rows the device computed
function orthogonality_loss(V::HIPBasis, k::Int)
    L = LowerTriangular(V.gram[1:k, 1:k])
    return norm(Matrix(Symmetric(Matrix(L), :L)) - I(k))
end

# ------------------------------------------------------------------ decomposition types
abstract type HIPTensorDecomposition{matT, T, U} <: TensorDecomposition{matT, T, U} end

const NMAX = Ref(0)    # capacity for the next constructor call (set by tensorkrylov! below)

for (Name, method, orth) in ((:HIPTensorArnoldi, TK_ARNOLDI, :Arnoldi),
                             (:HIPTensorLanczos, TK_LANCZOS, :Lanczos),
                             (:HIPTensorLanczosReorth, TK_LANCZOS_REORTH, :LanczosReorth))
    @eval begin
        mutable struct $Name{matT, T, U} <: HIPTensorDecomposition{matT, T, U}
            A::KronMat{matT, U}
            V::KronComp{HIPBasis}
            H::KronMat{Matrix{T}, U}
            orthonormalization::Type{$orth}
            dc::Union{Nothing, HIPDecomp}
            function $Name(A::KronMat{matT, U}) where {matT, U <: Instance}
                kmax = NMAX[] > 0 ? NMAX[] : size(first(A.M), 1)
                # host H_s is (kmax+2)^2 -- the reference's (n+1)^2 would not fit at n = 2^20
                H = KronMat{Matrix{Float64}, U}(fill(kmax + 2, length(A)))
                new{matT, Float64, U}(A, KronComp{HIPBasis}(HIPBasis[]), H, $orth, nothing)
            end
        end
        method_of(::$Name) = $method
    end
end

# tensorkrylov! needs nmax before the decomposition is built: record it, then run the
# package's own driver unchanged.  The signature is the reference's
# (src/tensor_krylov_method.jl:36-43) with argument 6 narrowed to the HIP types and argument 7
# typed exactly as there (mode::Type{<:Mode} = SilentMode): this method is then strictly more
# specific than the reference's in every argument.  (An untyped `mode` made the 7-argument
# call from the 6-argument default ambiguous -- more specific in argument 6, less in 7 -- and
# solve_tensorized_system, src/system.jl:73-79, raised a MethodError on the first solve.)
function tensorkrylov!(conv::ConvergenceData{T}, A::KronMat{matT, U}, b::KronProd{T}, tol::T, nmax::Int,
                       t::Type{<:HIPTensorDecomposition},
                       mode::Type{<:TensorKrylov.Mode} = TensorKrylov.SilentMode) where {matT, T, U <: Instance}
    NMAX[] = nmax
    try
        return invoke(tensorkrylov!, Tuple{ConvergenceData{T}, KronMat{matT, U}, KronProd{T}, T, Int,
                                           Type{<:TensorDecomposition}, Type{<:TensorKrylov.Mode}},
                      conv, A, b, tol, nmax, t, mode)
    finally
        NMAX[] = 0
    end
end

function apply_records!(td::HIPTensorDecomposition, rec::Matrix{Float64}, j::Int)
    kmax = td.dc.kmax
    for s in 1:td.dc.d
        r = @view rec[:, s]
        H = td.H.M[s]
        if j >= 0
            if td isa HIPTensorArnoldi
                H[1:j + 2, j + 1] .= r[1:j + 2]
            else
                reorth = td isa HIPTensorLanczosReorth && r[2kmax + 9] > 0
                if reorth                                   # src/orthogonal_bases.jl:123-131
                    H[1:j + 2, j + 1] .= r[1:j + 2]
                    H[1:max(j - 1, 0), j + 1] .= 0.0
                    β = H[j + 2, j + 1]
                else
                    H[j + 1, j + 1] = r[j + 1]
                    β = r[j + 2]
                end
                H[j + 2, j + 1] = β                         # update_subdiagonals!
                H[j + 1, j + 2] = β
            end
        end
        c = Int(r[2kmax + 6])
        if c >= 0
            td.V.M[s].btilde[c + 1] = r[2kmax + 5]
            r[2kmax + 10] > 0 && (td.V.M[s].gram[c + 1, 1:c + 1] .= r[kmax + 3:kmax + 3 + c])
        end
    end
end

# orthonormalize!(td, b): V[:,1] = b/|b| and step 1 (src/orthogonal_bases.jl:142-160)
function orthonormalize!(td::HIPTensorDecomposition, b::KronProd)
    ctx = context()
    kmax = size(td.H.M[1], 1) - 2
    cache = IdDict{Any, HIPMatrix}()
    mats = [get!(() -> HIPMatrix(ctx, As), cache, As) for As in td.A.M]
    td.dc = HIPDecomp(ctx, method_of(td), mats, b, kmax)
    td.V.M = [HIPBasis(td.dc, s, kmax + 1, zeros(kmax + 1), zeros(kmax + 1, kmax + 1)) for s in 1:length(mats)]
    apply_records!(td, records(td.dc, :init), -1)
    orthonormalize!(td, 1)
end

# orthonormalize!(td, k) for every factor in one batched launch set (src/orthogonal_bases.jl:162-180)
function orthonormalize!(td::HIPTensorDecomposition, k::Int)
    apply_records!(td, records(td.dc, :step, Cint(k - 1)), k - 1)
end

end # module
