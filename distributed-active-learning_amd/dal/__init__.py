"""dal -- MI355X-native active-learning query selection.

Drop-in replacement for the query-selection hot path of
dv66/Distributed-Active-Learning.  Modules keep the reference's script names:

  dal.uncertainty_sampling   final_thesis/uncertainty_sampling.py
  dal.density_weighting      final_thesis/density_weighting.py
  dal.cosine_similarity      final_thesis/cosine_similarity.py
  dal.similarity             final_thesis/similarity.py
  dal.forest                 the fitted RandomForest (MLlib trees) in device SoA form
  dal.parallel               the row-sharded multi-GPU path (RCCL over xGMI)

All arithmetic runs in hand-written HIP kernels for gfx950 (libdal.so, C ABI in
include/dal.h); importing this package does not require a GPU, calling it does.
"""
from .forest import Forest  # noqa: F401
from .luts import STRATEGIES, lut  # noqa: F401

__version__ = "0.1.0"
