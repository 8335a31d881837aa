"""``python -m nbdistributed_amd._native [--force]``: build libnbd_transport.so and libnbd_ops.so in-tree."""
import sys

from . import OPS_LIB, TRANSPORT_LIB, build_all

build_all(force="--force" in sys.argv)
print(TRANSPORT_LIB, OPS_LIB)
