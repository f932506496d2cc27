"""tkamd -- MI355X-native inner Krylov iteration of thbake/TensorKrylov.jl.

Host-side mirror of the reference's solver API (KroneckerMatrix, TensorizedSystem,
TensorArnoldi / TensorLanczos / TensorLanczosReorth, tensorkrylov!,
solve_tensorized_system) over the C-ABI library libtkhip.so (include/tk.h), whose
hand-written gfx950 kernels run the per-factor Krylov steps and V*Y.
"""
from ._lib import TKError, lib  # noqa: F401
from .compressed import (ApproximationData, CompressedNormBreakdown, SpectralData,  # noqa: F401
                         residualnorm, solve_compressed_system)
from .decompositions import (METHODS, Decomposition, Partition, TensorArnoldi,  # noqa: F401
                             TensorDecomposition, TensorLanczos, TensorLanczosReorth,
                             arnoldi_algorithm, isorthonormal, lanczos_algorithm,
                             orthogonality_loss)
from .device import Context, DeviceDecomposition, DeviceMatrix, unique_id  # noqa: F401
from .solver import solve_tensorized_system, tensorkrylov  # noqa: F401
from .structures import (ConvDiff, ConvergenceData, KroneckerMatrix, KruskalTensor,  # noqa: F401
                         kronecker_sum_matvec, kroneckervectorize,
                         Laplace, NonSymInstance, RandSparseSPD, SymInstance, TensorizedSystem,
                         as_csc, assemble_matrix, normalize_rhs, random_rhs)
