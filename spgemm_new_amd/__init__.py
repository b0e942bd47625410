"""spgemm_new_amd -- MI355X-native MaxK-GNN aggregation (forward SpGEMM + backward SSpMM).

Hot path: hand-written HIP kernels for gfx950 in ``csrc/maxk_spgemm.hip``,
reached through the C ABI ``include/maxk_spgemm.h`` (``lib/libmaxk_spgemm.so``).
Host-side mirrors of the reference surface:

* ``maxk_cuda_kernels``        cuda_kernel_bindings.cpp functional API
* ``spmm_kernels``             kernels/spmm_bindings.cpp class API
* ``models.MaxK`` / ``models.SpGEMMFunction``   utils/models.py:28-149
* ``direct_kernel_interface.DirectMaxKKernels`` direct_kernel_interface.py:24-382
* ``distributed``              1-D row partition + RCCL all-to-all-v halo
"""
from ._lib import LIB_PATH, MaxKError, load  # noqa: F401
from .ops import (MaxKGraph, cbsr_gather_records, cbsr_mask, cbsr_scatter, spgemm_forward,  # noqa: F401
                  spgemm_forward_records, spmm_dense, sspmm_backward, topk_cbsr, warp4_build)

__version__ = "0.1.0"
