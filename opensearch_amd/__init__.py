"""opensearch_amd — MI355X-native exact k-NN scoring for OpenSearch.

The product is libosknn.so (HIP kernels for gfx950 behind the C-ABI in include/osknn.h).  This
package holds its in-tree build, the ctypes binding, and the host-side mirror of the Lucene /
OpenSearch interfaces on the path (lucene.py, search.py, distributed.py).
"""
from . import _lib
from ._lib import OskError, device_count

__all__ = ["_lib", "OskError", "device_count"]
