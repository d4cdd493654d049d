"""Hand-written gfx950 HIP ops (csrc/kernels) behind thin Python wrappers."""
from .flat import FlatParams, flat_sgd_, sgd_update_, scale_by_count_, elastic_step_, add_, fill_
