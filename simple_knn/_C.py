"""`from simple_knn._C import distCUDA2` -- served by liblsr.so (langsplat_amd.knn)."""
from langsplat_amd.knn import dist_cuda2 as distCUDA2  # noqa: F401
