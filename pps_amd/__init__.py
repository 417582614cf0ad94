"""pps_amd: MI355X-native re-ID inference + retrieval path for PPS.

Hot path: ResNet-50 (stride-1 res5) + part-power-set heads as
hand-written gfx950 HIP kernels, and the query x gallery distance + rank +
mAP/CMC evaluation, behind the C ABI in include/pps_abi.h (libpps_hip.so).
"""
__version__ = '0.1.0'
