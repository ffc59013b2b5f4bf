"""dgen_amd -- MI355X-native engine for dGen's per-agent PV sizing & economics
hot path (financial_functions.calc_system_size_and_performance and the PySAM
Utilityrate5 / Cashloan / Battery work it drives), built for gfx950.

Layout:
  csrc/dgen_hip.hip   hand-written HIP kernels + the C-ABI (include/dgen_hip.h)
  _lib.py             ctypes binding (fails loudly: no CPU fallback)
  engine.py           resident tables + batched sizing on one GPU
  tariff.py           host tariff compiler (normalize_tariff / process_tariff)
  columnar.py         agent rows -> SoA columns, rate-switch candidates
  financial_functions.py  drop-in for the reference module's hot-path API
  synth.py            synthetic populations
  dist.py             agent sharding across ranks + per-(state, sector) totals
"""
__version__ = "0.1.0"
