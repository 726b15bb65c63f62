"""ctypes binding of libkhst.so (include/khst.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (hipcc,
--offload-arch=gfx950).  There is no fallback: if the library is missing or no
device is usable, every entry point raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KHST_LIB_AB") or os.path.join(_HERE, "libkhst.so")  # KHST_LIB_AB: an A/B build (measurement only)

KH_OK = 0
KH_EINVAL = -1
KH_ENOMEM = -2
KH_EDEVICE = -3
KH_ENODE = -4
KH_EINTERNAL = -5
KH_ENOSPC = -6
KH_HASH_KEYS = 0x1
KH_EMIT_NODES = 0x2
KH_SHARD_RCCL = 0x4  # kh_trie_root_sharded: the RCCL exchange even when a device repeats (tests' loopback)
KH_NO_TRIE = 0xFFFFFFFF

# every symbol include/khst.h declares
EXPORTS = (
    "kh_last_error", "kh_version", "kh_device_count", "kh_kec256_batch", "kh_trie_root",
    "kh_trie_roots_segmented", "kh_trie_root_nodes", "kh_ctx_create", "kh_ctx_destroy", "kh_ctx_set_stream",
    "kh_dev_kec256_batch", "kh_dev_trie_build", "kh_dev_trie_build_ev", "kh_fold_root16", "kh_dev_synth_accounts", "kh_dev_hash_keys",
    "kh_dev_partition", "kh_dev_partition_ev", "kh_dev_hash_partition_ev", "kh_trie_open", "kh_trie_apply", "kh_trie_emit_nodes", "kh_trie_size", "kh_trie_free",
    "kh_verify_nodes", "kh_trie_open_host", "kh_trie_apply_host", "kh_forest_open", "kh_forest_apply",
    "kh_forest_apply_host", "kh_block_commit", "kh_forest_last_roots", "kh_trie_open_nodes",
    "kh_trie_open_nodes_host", "kh_trie_roots_varkeys", "kh_list_roots",
    "kh_trie_root_sharded", "kh_block_commit_host", "kh_dev_list_roots", "kh_trie_get", "kh_trie_get_host",
    "kh_dev_synth_storage", "kh_trie_roots_segmented_sharded", "kh_trie_savepoint", "kh_trie_rollback",
    "kh_trie_release", "kh_trie_savepoint_depth", "kh_trie_root_of", "kh_trie_root_of_host", "kh_trie_copy",
    "kh_verify_nodes_packed", "kh_trie_usage", "kh_trie_compact",
)


class KhError(RuntimeError):
    """Base error of the C ABI (status code in .code)."""

    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class MPTException(KhError):
    """KH_EINVAL: the analogue of MerklePatriciaTrie.MPTException / RLPException
    (MerklePatriciaTrie.scala:46, rlp/package.scala:11)."""


class MPTNodeMissingException(KhError):
    """KH_ENODE (MerklePatriciaTrie.scala:47)."""


class DeviceError(KhError):
    """KH_EDEVICE / KH_ENOMEM: the GPU path failed."""


class KhTrieUsage(ctypes.Structure):
    """kh_trie_usage_t: a resident handle's records, value heap and HBM (include/khst.h)."""
    _fields_ = [(f, ctypes.c_uint64) for f in
                ("records", "live_records", "heap_bytes", "live_heap_bytes", "map_slots", "hbm_bytes")]


class KhStats(ctypes.Structure):
    _fields_ = [
        ("n_inputs", ctypes.c_uint64), ("n_leaves", ctypes.c_uint64), ("n_branches", ctypes.c_uint64),
        ("n_extensions", ctypes.c_uint64), ("n_inline", ctypes.c_uint64), ("n_node_hashes", ctypes.c_uint64),
        ("n_node_perms", ctypes.c_uint64), ("n_key_perms", ctypes.c_uint64), ("arena_bytes", ctypes.c_uint64),
        ("n_levels", ctypes.c_uint32), ("full_sort", ctypes.c_uint32), ("t_total_ms", ctypes.c_double),
        ("t_keys_ms", ctypes.c_double), ("t_sort_ms", ctypes.c_double), ("t_topo_ms", ctypes.c_double),
        ("t_leaf_ms", ctypes.c_double), ("t_branch_ms", ctypes.c_double), ("reserved0", ctypes.c_uint32),
        ("reserved", ctypes.c_uint32),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


_lib = None


def lib():
    """Load libkhst.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    # torch ships its own libamdhip64.so.7 (same soname as /opt/rocm's): whichever is
    # loaded first serves the whole process.  Load torch's first so torch (the HBM
    # allocator) and libkhst share one HIP runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} not built: run __graft_entry__.build() (hipcc --offload-arch=gfx950)")
    L = ctypes.CDLL(LIB_PATH)
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.kh_last_error.restype = ctypes.c_char_p
    L.kh_version.restype = ctypes.c_char_p
    L.kh_device_count.restype = i32
    L.kh_kec256_batch.argtypes = [vp, vp, u64, vp]
    L.kh_trie_root.argtypes = [vp, u32, vp, vp, u64, u32, vp, vp]
    L.kh_trie_roots_segmented.argtypes = [vp, u32, vp, vp, vp, u64, u32, vp, vp]
    L.kh_trie_root_nodes.argtypes = [vp, u32, vp, vp, u64, u32, vp, vp, u64, vp, u64, vp, vp, vp, vp]
    L.kh_ctx_create.argtypes = [i32, ctypes.POINTER(vp)]
    L.kh_ctx_destroy.argtypes = [vp]
    L.kh_ctx_set_stream.argtypes = [vp, vp]
    L.kh_dev_kec256_batch.argtypes = [vp, vp, vp, u64, vp]
    L.kh_dev_trie_build.argtypes = [vp, vp, u32, vp, vp, u64, vp, u64, u32, u32, vp, vp, vp, vp]
    L.kh_dev_trie_build_ev.argtypes = [vp, vp, vp, u32, vp, vp, u64, vp, u64, u32, u32, vp, vp, vp, vp]
    L.kh_fold_root16.argtypes = [vp, vp, vp, vp]
    L.kh_dev_synth_accounts.argtypes = [vp, u32, u64, u64, vp, vp, vp]
    L.kh_dev_hash_keys.argtypes = [vp, vp, u32, u64, vp]
    L.kh_dev_partition.argtypes = [vp, vp, vp, vp, u64, u32, vp, vp, vp, vp, vp]
    L.kh_dev_partition_ev.argtypes = [vp, vp, vp, vp, vp, u64, u32, vp, vp, vp, vp, vp]
    L.kh_dev_hash_partition_ev.argtypes = [vp, vp, vp, u32, vp, vp, u64, u32, vp, vp, vp, vp, vp]
    L.kh_trie_open.argtypes = [vp, vp, u32, vp, vp, u64, u32, vp, ctypes.POINTER(vp)]
    L.kh_trie_apply.argtypes = [vp, vp, vp, vp, u64, vp, u64, u32, u32, vp, vp]
    L.kh_trie_emit_nodes.argtypes = [vp, vp, u64, vp, u64, vp, vp, vp]
    L.kh_trie_size.argtypes = [vp, ctypes.POINTER(u64)]
    L.kh_trie_free.argtypes = [vp]
    L.kh_verify_nodes.argtypes = [vp, vp, u64, vp, vp, u64, vp, vp, vp, vp, vp, vp]
    L.kh_trie_open_host.argtypes = [vp, u32, vp, vp, u64, u32, vp, ctypes.POINTER(vp)]
    L.kh_trie_apply_host.argtypes = [vp, vp, vp, vp, u64, vp, u64, u32, u32, vp, vp]
    L.kh_forest_open.argtypes = [vp, u32, ctypes.POINTER(vp)]
    L.kh_forest_apply.argtypes = [vp, vp, vp, vp, vp, u64, vp, vp, u64, u32, vp, vp, u64, vp, vp]
    L.kh_forest_apply_host.argtypes = [vp, vp, vp, vp, vp, u64, vp, vp, u64, u32, vp, vp, u64, vp, vp]
    L.kh_forest_last_roots.argtypes = [vp, vp, vp, u64, vp]
    L.kh_trie_open_nodes.argtypes = [vp, vp, vp, vp, u64, u32, vp, ctypes.POINTER(vp)]
    L.kh_trie_open_nodes_host.argtypes = [vp, vp, vp, u64, u32, vp, ctypes.POINTER(vp)]
    L.kh_block_commit.argtypes = [vp, vp, vp, vp, vp, vp, u64, vp, vp, u64, u32, vp, vp, vp, vp, u64, vp, u64, u32,
                                  vp, vp]
    L.kh_trie_roots_varkeys.argtypes = [vp, vp, vp, vp, vp, u64, vp, vp]
    L.kh_list_roots.argtypes = [vp, vp, vp, u64, vp, vp]
    L.kh_trie_root_sharded.argtypes = [vp, i32, vp, u32, vp, vp, u64, u32, vp, vp]
    L.kh_block_commit_host.argtypes = L.kh_block_commit.argtypes
    L.kh_dev_list_roots.argtypes = [vp, vp, vp, vp, u64, vp, vp]
    L.kh_trie_get.argtypes = [vp, vp, vp, u32, u64, vp, u64, vp, vp, ctypes.POINTER(u64)]
    L.kh_dev_synth_storage.argtypes = [vp, u32, u64, u64, vp, ctypes.POINTER(u64), ctypes.POINTER(u64), vp, vp, vp, vp]
    L.kh_trie_roots_segmented_sharded.argtypes = [vp, i32, vp, u32, vp, vp, vp, u64, u32, vp, vp]
    L.kh_trie_get_host.argtypes = [vp, vp, vp, u32, u64, vp, u64, vp, vp, ctypes.POINTER(u64)]
    L.kh_trie_savepoint.argtypes = [vp, ctypes.POINTER(u32)]
    L.kh_trie_rollback.argtypes = [vp]
    L.kh_trie_release.argtypes = [vp]
    L.kh_trie_savepoint_depth.argtypes = [vp, ctypes.POINTER(u32)]
    L.kh_trie_root_of.argtypes = L.kh_trie_apply.argtypes
    L.kh_trie_root_of_host.argtypes = L.kh_trie_apply_host.argtypes
    L.kh_trie_copy.argtypes = [vp, ctypes.POINTER(vp)]
    L.kh_trie_usage.argtypes = [vp, ctypes.POINTER(KhTrieUsage)]
    L.kh_trie_compact.argtypes = [vp, ctypes.POINTER(KhTrieUsage)]
    L.kh_verify_nodes_packed.argtypes = [vp, vp, u64, vp, vp, u64, vp, vp, vp, vp, vp, vp, u64, ctypes.POINTER(u64)]
    for name in EXPORTS:
        fn = getattr(L, name)
        if fn.restype is ctypes.c_int or name not in ("kh_last_error", "kh_version"):
            if name not in ("kh_last_error", "kh_version"):
                fn.restype = i32
    _lib = L
    return L


def check(rc):
    if rc == KH_OK:
        return
    msg = lib().kh_last_error().decode(errors="replace")
    if rc == KH_EINVAL:
        raise MPTException(rc, msg)
    if rc == KH_ENODE:
        raise MPTNodeMissingException(rc, msg)
    if rc in (KH_EDEVICE, KH_ENOMEM):
        raise DeviceError(rc, msg)
    raise KhError(rc, msg)
