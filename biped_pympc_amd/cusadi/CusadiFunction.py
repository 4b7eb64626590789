"""Drop-in ``CusadiFunction`` (reference ``biped_pympc/cusadi/src/CusadiFunction.py:6-117``).

Same constructor, attributes and methods -- ``evaluate(inputs)``, ``outputs_sparse[i]``,
``getDenseOutput(i)``, ``eval_time``, ``checkInputDimensions`` -- bound through ctypes to the same
``float evaluate(const double**, double*, double**, int)`` symbol of ``lib<fn.name()>.so``, now a
thin library over the hand-written HIP kernels (``include/srbd_mpc.h``). Differences, all
deliberate:
  * ``fn_casadi`` is a ``biped_pympc_amd.cusadi.Function`` descriptor (no CasADi dependency);
  * a failing kernel raises ``RuntimeError`` with the library's message instead of the reference's
    ``exit(code)`` inside ``gpuErrchk`` (``generateCUDACode.py:106-112``);
  * the device pointer tables are refreshed with one host->device copy instead of one per element,
    and ``getDenseOutput`` is one scatter kernel over a cached index map (same results);
  * ``outputs_dense`` is allocated lazily, entry by entry, when it is read: the reference allocates
    a zeroed ``(B, size1, size2)`` tensor per output in ``_setup`` (``CusadiFunction.py:77-81``)
    that nothing ever writes (``getDenseOutput`` returns a new tensor), which for ``qp_former`` at
    B = 4096, N = 10 is 4.25 GB of HBM held for nothing. Reading ``outputs_dense[i]`` still gives
    that zeroed tensor.
As in the reference, the caller's tensors are used in place through ``data_ptr()`` and their
strides are NOT consulted: pass contiguous ``(num_instances, nnz_in[i])`` FP64 CUDA tensors.
"""
from __future__ import annotations

import ctypes
import os
import sys

import torch

from biped_pympc_amd.build import LIB_DIR, build_dropin
from biped_pympc_amd.controller import dense_scatter, inverse_index


class _LazyDenseOutputs:
    """``outputs_dense`` of a CusadiFunction: a sequence of zeroed ``(B, size1_out(i), size2_out(i))``
    FP64 tensors, each allocated on its first read and then kept (as the reference's list is)."""

    def __init__(self, fn, num_instances: int, device):
        self._fn, self._B, self._device = fn, num_instances, device
        self._cache = {}

    def __len__(self):
        return self._fn.n_out()

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[k] for k in range(*i.indices(len(self)))]
        if i < 0:
            i += len(self)
        if not 0 <= i < len(self):
            raise IndexError(i)
        if i not in self._cache:
            self._cache[i] = torch.zeros((self._B, self._fn.size1_out(i), self._fn.size2_out(i)),
                                         device=self._device, dtype=torch.double)
        return self._cache[i]

    def __iter__(self):
        return (self[k] for k in range(len(self)))

    @property
    def allocated(self) -> list[int]:
        """Indices of the entries read so far (the others hold no device memory)."""
        return sorted(self._cache)


class CusadiFunction:
    # Public variables:
    fn_casadi = None
    fn_name = None
    num_instances = 0
    inputs_sparse = []
    outputs_sparse = []
    outputs_dense = []

    # Private variables:
    _device = "cuda"

    def __init__(self, fn_casadi, num_instances: int):
        assert torch.cuda.is_available()
        lib_filepath = os.path.join(LIB_DIR, f"lib{fn_casadi.name()}.so")
        if not os.path.exists(lib_filepath):
            build_dropin(fn_casadi.kind, fn_casadi.horizon, fn_casadi.n_iter)
        self.fn_casadi = fn_casadi
        self.fn_name = fn_casadi.name()
        self.num_instances = int(num_instances)
        self._fn_library = ctypes.CDLL(lib_filepath)
        self._fn_library.evaluate.restype = ctypes.c_float
        self._fn_library.evaluate.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_int]
        self._core = ctypes.CDLL(os.path.join(LIB_DIR, "libsrbd_mpc.so"))
        self._core.srbd_last_error.restype = ctypes.c_char_p
        self._dense_index = {}
        self.eval_time = 0.0
        print("Loaded CasADi function: ", self.fn_casadi)
        print("Loaded library: ", self._fn_library)
        self._setup()

    def evaluate(self, inputs):
        self._clearTensors()
        self._prepareInputTensor(inputs)
        t = self._fn_library.evaluate(self._fn_input, self._fn_work, self._fn_output,
                                      self.num_instances)
        if t < 0:
            raise RuntimeError(f"{self.fn_name}: {self._core.srbd_last_error().decode(errors='replace')}")
        self.eval_time = t

    def getDenseOutput(self, out_idx=None):
        """(B, size1, size2) dense output, scattered by one HIP kernel from the nonzeros through a
        cached dense -> nonzero index map (the reference builds a COO tensor from Python lists
        and calls .to_dense() on every call, CusadiFunction.py:49-58)."""
        fn = self.fn_casadi
        s1, s2 = fn.size1_out(out_idx), fn.size2_out(out_idx)
        if out_idx not in self._dense_index:
            rows, cols = fn.sparsity_out(out_idx).get_triplet()
            self._dense_index[out_idx] = inverse_index(rows, cols, (s1, s2), self._device)
        return dense_scatter(self.outputs_sparse[out_idx].reshape(self.num_instances, -1),
                             self._dense_index[out_idx], (s1, s2))

    def checkInputDimensions(self, inputs):
        """Shape check of every input (the reference runs one CPU CasADi call, :60-67)."""
        fn = self.fn_casadi
        ok = len(inputs) == fn.n_in() and all(
            t.numel() == self.num_instances * fn.nnz_in(i) and t.dtype == torch.double
            for i, t in enumerate(inputs))
        if ok:
            print("Input check successful. Tensor dimensions are correct for inputs.")
        else:
            print("Error in input dimensions. Exiting...")
            sys.exit(1)

    # ! Private methods:
    def _setup(self):
        fn = self.fn_casadi
        B = self.num_instances
        self._input_tensors = [torch.zeros((B, fn.nnz_in(i)), device=self._device, dtype=torch.double)
                               for i in range(fn.n_in())]
        self._output_tensors = [torch.zeros(B, fn.nnz_out(i), device=self._device, dtype=torch.double)
                                for i in range(fn.n_out())]
        self._output_tensors_dense = _LazyDenseOutputs(fn, B, self._device)
        self._work_tensor = torch.zeros((B, max(fn.sz_w(), 1)), device=self._device, dtype=torch.double)
        self._input_ptrs = torch.zeros(fn.n_in(), device=self._device, dtype=torch.int64)
        self._output_ptrs = torch.tensor([t.data_ptr() for t in self._output_tensors],
                                         device=self._device, dtype=torch.int64)
        self._fn_input = ctypes.c_void_p(self._input_ptrs.data_ptr())
        self._fn_output = ctypes.c_void_p(self._output_ptrs.data_ptr())
        self._fn_work = ctypes.c_void_p(self._work_tensor.data_ptr())
        self.inputs_sparse = self._input_tensors
        self.outputs_sparse = self._output_tensors
        self.outputs_dense = self._output_tensors_dense

    def _prepareInputTensor(self, inputs):
        for i in range(self.fn_casadi.n_in()):
            self._input_tensors[i] = inputs[i]
        self._input_ptrs.copy_(torch.tensor([t.data_ptr() for t in self._input_tensors],
                                            dtype=torch.int64))
        self.inputs_sparse = self._input_tensors

    def _clearTensors(self):
        for t in self._output_tensors:
            t.zero_()
        self._work_tensor.zero_()
