"""``python -m nbdistributed_amd._native [--force]``: build libnbd_transport.so and libnbd_ops.so in-tree."""
import sys

from . import build_all, build_ops, build_transport

build_all(force="--force" in sys.argv)
print(build_transport(), build_ops())
