"""CusADi-compatible runtime surface (reference ``biped_pympc/cusadi/src/__init__.py:3-18``).

``CASADI_FUNCTION_DIR`` holds the function descriptors (the reference's ``.casadi`` artefacts);
``CUSADI_FUNCTION_DIR`` holds the ``lib<name>.so`` libraries exporting ``evaluate``.
"""
import os

from biped_pympc_amd.build import LIB_DIR
from biped_pympc_amd.cusadi.CusadiFunction import CusadiFunction
from biped_pympc_amd.cusadi.function import (FUNCTION_DIR, Function, Sparsity, pdipm_function,
                                             qp_former_function)

CUSADI_ROOT_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASADI_FUNCTION_DIR = FUNCTION_DIR
CUSADI_FUNCTION_DIR = LIB_DIR

__all__ = ["CusadiFunction", "Function", "Sparsity", "qp_former_function", "pdipm_function",
           "CASADI_FUNCTION_DIR", "CUSADI_FUNCTION_DIR", "CUSADI_ROOT_DIR"]
