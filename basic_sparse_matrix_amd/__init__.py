"""basic_sparse_matrix_amd -- MI355X-native (gfx950) implementation of the
CSR x dense multiply and Cholesky/solve hot path of the Rust crate
jamieapps101/Basic_Sparse_Matrix, behind the same Csr/Dense/solve API.

Host logic (construction, accessors) is Python; every compute method runs
hand-written HIP kernels through the C-ABI in include/bsm.h
(libbsm_hip.so). See DESIGN.md.
"""

from .dense import Dense
from .dense_static import DenseS
from .multi import set_gpus
from .solver import backward_substitution, forward_substitution, solve
from .sparse import COO, COOEntry, Csr, CsrEntry
from .util import GetDims, MatDim, MatErr, MatErrKind, Panic

__all__ = [
    "set_gpus",
    "COO",
    "COOEntry",
    "Csr",
    "CsrEntry",
    "Dense",
    "DenseS",
    "GetDims",
    "MatDim",
    "MatErr",
    "MatErrKind",
    "Panic",
    "solve",
    "forward_substitution",
    "backward_substitution",
]
