"""Fast-sync NodeData verification on the GPU.

Mirror of NodeDatasRequest.processResponse (khipu-eth/.../blockchain/sync/
package.scala:81-125) over kh_verify_nodes: every value a peer returned is
kec256'd, matched against the requested hashes, and a matched trie node is decoded
with PV63's MptNode rules (network/p2p/messages/PV63.scala:96-127) to list the
children still to download (getStateNodeChildren / getContractMptNodeChildren,
sync/package.scala:127-165).  The hashing and decoding run in libkhst's HIP kernel;
this module only assembles the response lists in the reference's order.
"""
import ctypes
from collections import namedtuple

import numpy as np

from ._lib import check, lib

# NodeHash kinds (sync/package.scala NodeHash subclasses)
STATE_NODE, STORAGE_ROOT, CONTRACT_NODE, EVMCODE = 0, 1, 2, 3
KIND_NAMES = {STATE_NODE: "StateMptNodeHash", STORAGE_ROOT: "StorageRootHash",
              CONTRACT_NODE: "ContractStorageMptNodeHash", EVMCODE: "EvmcodeHash"}
STATUS_MSG = {1: "Cannot decode NodeData", 2: "unexpected value in node", 3: "Cannot decode Account",
              4: "malformed RLP"}

NodeHash = namedtuple("NodeHash", "hash kind")
NodeDatasResponse = namedtuple("NodeDatasResponse", "peer_id n_downloaded_nodes remaining_hashes children_hashes "
                                                    "received_accounts received_storages received_evmcodes")


class NodeDataError(RuntimeError):
    """The reference throws a RuntimeException from MptNode decoding."""


def verify_nodes(values, requests):
    """kh_verify_nodes over host data.  values: list of bytes; requests: list of
    NodeHash.  Returns (hashes [n,32], match [n], status [n], children list per value)."""
    n = len(values)
    blob = b"".join(values)
    data = np.frombuffer(blob + b"\0" * 16, np.uint8)
    off = np.zeros(n + 1, np.uint64)
    if n:
        off[1:] = np.cumsum([len(v) for v in values])
    nreq = len(requests)
    req = np.frombuffer(b"".join(r.hash for r in requests) + b"\0" * 32, np.uint8)
    kind = np.array([r.kind for r in requests] + [0], np.uint8)
    hh = np.zeros((max(n, 1), 32), np.uint8)
    match = np.zeros(max(n, 1), np.int64)
    status = np.zeros(max(n, 1), np.uint8)
    nchild = np.zeros(max(n, 1), np.uint8)
    child = np.zeros((max(n, 1), 16, 32), np.uint8)
    ckind = np.zeros((max(n, 1), 16), np.uint8)
    check(lib().kh_verify_nodes(data.ctypes.data, off.ctypes.data, n, req.ctypes.data, kind.ctypes.data, nreq,
                                hh.ctypes.data, match.ctypes.data, status.ctypes.data, nchild.ctypes.data,
                                child.ctypes.data, ckind.ctypes.data))
    kids = [[NodeHash(child[i, j].tobytes(), int(ckind[i, j])) for j in range(int(nchild[i]))] for i in range(n)]
    return hh[:n], match[:n], status[:n], kids


class NodeDatasRequest:
    """sync/package.scala:77-125 (the GPU does the hashing and the node decoding)."""

    def __init__(self, peer_id, request_node_hashes):
        self.peer_id = peer_id
        self.request_node_hashes = list(request_node_hashes)

    def process_response(self, values):
        if not values:
            return None
        hh, match, status, kids = verify_nodes(values, self.request_node_hashes)
        received, children, accounts, storages, codes = set(), [], [], [], []
        for i, v in enumerate(values):
            m = int(match[i])
            if m < 0:
                continue
            x = self.request_node_hashes[m]
            if status[i]:
                raise NodeDataError(STATUS_MSG.get(int(status[i]), "decode error"))
            received.add(x)
            if x.kind == STATE_NODE:
                children += kids[i]
                accounts.insert(0, (x.hash, v))
            elif x.kind in (STORAGE_ROOT, CONTRACT_NODE):
                children += kids[i]
                storages.insert(0, (x.hash, v))
            else:
                codes.insert(0, (x.hash, v))
        remaining = [h for h in self.request_node_hashes if h not in received]
        return NodeDatasResponse(self.peer_id, len(received), remaining, children, accounts, storages, codes)
