from .buckets import GradBucketer
from .comm import all_reduce_, barrier, broadcast_, init_process_group, is_dist, rank, world_size
from .strategy import (CentralStorageStrategy, MirroredStrategy, OneDeviceStrategy, Strategy,
                       default_strategy)

__all__ = ["GradBucketer", "all_reduce_", "barrier", "broadcast_", "init_process_group", "is_dist",
           "rank", "world_size", "CentralStorageStrategy", "MirroredStrategy", "OneDeviceStrategy",
           "Strategy", "default_strategy"]
