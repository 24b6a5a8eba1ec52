"""addapt_amd -- MI355X-native engine for addapt's fold -> score -> accept hot path.

The HIP kernels and the C ABI live in ``addapt_amd/_lib/libaddapt_gpu.so``
(sources in ``addapt_amd/csrc``); ``addapt_amd.native`` is the ctypes binding
and ``addapt_amd.workloads`` builds the BASELINE.json inputs.  The C++ mirror of
the reference's Device / ScoreFunction / MonteCarlo API is
``addapt_amd/_lib/libaddapt_host.so`` (headers in ``include/addapt/``).
"""
from . import native  # noqa: F401

__all__ = ["native"]
