"""uwvk — batched PoseUKF / VelocityUKF on MI355X (gfx950).

Python host layer over the C ABI in include/uwvk.h (libuwvk.so).  The compute
path is HIP only: without the library or a gfx950 device the engine raises.
"""
