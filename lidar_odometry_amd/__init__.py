"""lidar_odometry_amd — MI355X-native point-to-plane ICP registration core.

Drop-in for the Gauss-Newton scan-to-map step of SiarheiHerasiuta/lidar_odometry
(IterativeClosestPointOptimizer::optimize + VoxelMap::GetSurfelAtPoint + PKO), implemented as HIP kernels
for gfx950 behind the C ABI in ``include/lo_icp.h`` (``liblo_icp.so``).
"""
from ._lib import LIB_PATH, lib, pinned_empty  # noqa: F401
from .icp import (AdaptiveMEstimatorConfig, BatchOptimizer, BatchResult, ICPConfig,  # noqa: F401
                  IterativeClosestPointOptimizer, MapGeometry, OptimizationStats)

__all__ = ["IterativeClosestPointOptimizer", "BatchOptimizer", "BatchResult", "ICPConfig", "AdaptiveMEstimatorConfig", "MapGeometry",
           "OptimizationStats", "lib", "LIB_PATH"]
