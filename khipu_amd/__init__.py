"""khipu_amd — MI355X batch state-root engine for khipu's Merkle-Patricia trie.

The product is libkhst.so (HIP kernels for gfx950 behind the C ABI in
include/khst.h).  This package holds its ctypes binding, the host-side mirror
of the reference's trie/crypto entry points, the value codecs, and the
multi-GPU driver.
"""
from ._lib import (DeviceError, KhError, KhStats, MPTException, MPTNodeMissingException, KH_HASH_KEYS, LIB_PATH,
                   lib)
from .trie import EMPTY_TRIE_HASH, MerklePatriciaTrie, kec256, kec256_batch, trie_root, trie_root_nodes, trie_roots

__all__ = [
    "DeviceError", "KhError", "KhStats", "MPTException", "MPTNodeMissingException", "KH_HASH_KEYS", "LIB_PATH", "lib",
    "EMPTY_TRIE_HASH", "MerklePatriciaTrie", "kec256", "kec256_batch", "trie_root", "trie_root_nodes", "trie_roots",
]
