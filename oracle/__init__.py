"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the CPU restatement (oracle/gmm_oracle.c).

Parity status: UNPINNED (see gmm_oracle.h).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this package.
"""
from .oracle import (OracleFloat, OracleFloatSum, OraclePresel, OracleSimd, libc_rand_sequence, batch_fast_score, batch_float_score, batch_int_prepare, batch_int_score, build,
                     constant_weight, quantize_array,
                     float_distance, gauss_log_norm, inverse_sqrt, load, quantization_scaling_factor, quantize,
                     simd_final_score)

__all__ = ["OracleFloat", "OracleFloatSum", "OraclePresel", "OracleSimd", "libc_rand_sequence", "batch_fast_score", "batch_float_score", "batch_int_prepare", "batch_int_score", "build",
           "constant_weight", "quantize_array",
           "float_distance", "gauss_log_norm", "inverse_sqrt", "load", "quantization_scaling_factor", "quantize",
           "simd_final_score"]
