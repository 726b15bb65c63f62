/*
 * khst — MI355X batch state-root engine for khipu's Merkle-Patricia trie.
 * C ABI of libkhst.so (khipu_amd/libkhst.so).  Plain pointers and sizes only.
 *
 * Every entry point replaces a reference interface on the state-root path
 * (paths relative to /root/reference/khipu-base/src/main/scala/khipu/ unless
 * they start with khipu-eth/):
 *
 *   kh_kec256_batch         crypto.kec256(Array[Byte]*)            crypto/package.scala:37-47
 *                           (one call per message today; here one call per batch,
 *                           e.g. NodeDatasRequest.processResponse,
 *                           khipu-eth/.../blockchain/sync/package.scala:88-90)
 *   kh_trie_root            foldLeft(put) + rootHash over a fresh trie:
 *                           MerklePatriciaTrie.put/rootHash  trie/MerklePatriciaTrie.scala:78,157-281
 *                           as driven by TrieAccounts.flush   khipu-eth/.../ledger/TrieAccounts.scala:22-28
 *                           and GenesisDataLoader             khipu-eth/.../blockchain/data/GenesisDataLoader.scala:139-147
 *   kh_trie_roots_segmented many independent tries (TrieStorage.flush per contract,
 *                           khipu-eth/.../ledger/TrieStorage.scala:52-60; BlockWorldState.scala:243-252)
 *   kh_trie_root_nodes      rootHash + the write-back node set of MerklePatriciaTrie.changes/persist
 *                           (MerklePatriciaTrie.scala:491-516,544-554 -> NodeStorage.update,
 *                           khipu-eth/.../storage/NodeStorage.scala:16-19)
 *   kh_trie_roots_varkeys   generic unhashed keys of any length <= 32 B, branch values
 *   kh_list_roots           transactions / receipts roots (MptListValidator.scala:15-46)
 *   kh_trie_root_sharded    the same root computed from per-GPU top-nibble shards
 *
 * Semantics shared by every trie entry point:
 *   - input i is a put(key_i, value_i); later inputs overwrite earlier ones with the
 *     same key (the foldLeft order of TrieAccounts.flush);
 *   - keys are `klen` bytes each; with KH_HASH_KEYS the trie key is kec256(key)
 *     (Address.hashedAddressEncoder, khipu-eth/.../domain/Address.scala:15-17;
 *     trie/package.scala:34-36), otherwise klen must be 32 (already keccak'd);
 *   - values are the serialised bytes (vSerializer.toBytes), packed: value i is
 *     vals[voff[i] .. voff[i+1]);
 *   - the root is kec256(encoding of the root node) even when that encoding is
 *     shorter than 32 bytes (MerklePatriciaTrie.scala:169); an empty trie has root
 *     EMPTY_TRIE_HASH = kec256(0x80) (trie/package.scala:41).
 *
 * Errors: int status; message via kh_last_error() (thread-local).  KH_EDEVICE means
 * the GPU path failed; the caller decides what to do (there is no silent fallback).
 * Threading: every call is reentrant.  Host entry points share one lazily created
 * device context per device; every call that uses a context holds its (recursive) mutex
 * for the call, and every call on a resident handle (kh_trie / forest) holds the mutex of
 * the context the handle was opened on, so calls on handles of one context from many
 * threads are serialised (a thread reading one handle's write-back set waits for another
 * thread's commit on the same context to finish, never for anything else).  A commit
 * whose in-flight tail (records, anchor map) fails leaves its handle refusing every call
 * but kh_trie_rollback (to a savepoint opened before it) and kh_trie_free.
 */
#ifndef KHST_H
#define KHST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KH_OK 0
#define KH_EINVAL -1     /* bad argument (RLPException / MPTException analogue) */
#define KH_ENOMEM -2     /* device allocation failed */
#define KH_EDEVICE -3    /* HIP runtime / kernel failure, or no device */
#define KH_ENODE -4      /* missing node (MPTNodeMissingException analogue) */
#define KH_EINTERNAL -5
#define KH_ENOSPC -6     /* caller's output buffer too small; required sizes returned */

/* flags */
#define KH_HASH_KEYS 0x1u   /* trie key = kec256(input key) */
#define KH_EMIT_NODES 0x2u  /* resident tries: keep each commit's write-back set (kh_trie_emit_nodes) */
#define KH_SHARD_RCCL 0x4u  /* kh_trie_root_sharded: exchange over RCCL even when a device repeats (needs a
                               communicator that accepts repeats, such as the tests' loopback) */
typedef struct kh_ctx kh_ctx;
#define KH_NO_TRIE 0xFFFFFFFFu  /* kh_block_commit: an account upsert without a storage trie */

typedef struct kh_stats {
  uint64_t n_inputs;       /* puts received */
  uint64_t n_leaves;       /* distinct keys (leaves) */
  uint64_t n_branches;
  uint64_t n_extensions;
  uint64_t n_inline;       /* nodes embedded in their parent (encoding < 32 B) */
  uint64_t n_node_hashes;  /* Keccak-256 of node encodings >= 32 B, plus one per root */
  uint64_t n_node_perms;   /* Keccak-f[1600] permutations spent on node encodings */
  uint64_t n_key_perms;    /* permutations spent hashing keys (KH_HASH_KEYS) */
  uint64_t arena_bytes;    /* bytes of node RLP produced */
  uint32_t n_levels;       /* bottom-up branch levels launched */
  uint32_t full_sort;      /* 1 if the 64-bit-prefix sort had ties and a full-key sort ran */
  double t_total_ms;       /* device time of the whole build (HIP events) */
  double t_keys_ms;        /* key hashing */
  double t_sort_ms;        /* radix sort + gather + dedup */
  double t_topo_ms;        /* LCP + topology */
  double t_leaf_ms;        /* leaf encode + hash */
  double t_branch_ms;      /* all branch levels */
  uint32_t reserved0;      /* 0 (kept for the layout the JNI shim and ctypes mirror) */
  uint32_t reserved;
} kh_stats;

const char* kh_last_error(void);
const char* kh_version(void);
int kh_device_count(void);

/* Batched kec256 over n messages packed as data[off[i] .. off[i+1]).  Host buffers. */
int kh_kec256_batch(const uint8_t* data, const uint64_t* off, uint64_t n, uint8_t* out32);

/* Root of the trie holding puts (key_i, val_i), i < n.  Host buffers. */
int kh_trie_root(const uint8_t* keys, uint32_t klen, const uint8_t* vals, const uint64_t* voff, uint64_t n,
                 uint32_t flags, uint8_t root32[32], kh_stats* stats);

/* nseg independent tries; trie s holds inputs seg_off[s] .. seg_off[s+1).  roots32: nseg*32 bytes. */
int kh_trie_roots_segmented(const uint8_t* keys, uint32_t klen, const uint8_t* vals, const uint64_t* voff,
                            const uint64_t* seg_off, uint64_t nseg, uint32_t flags, uint8_t* roots32,
                            kh_stats* stats);

/* Tries over variable-length unhashed keys of 0..32 bytes (key i = keys[koff[i] ..
 * koff[i+1])): a key that is a prefix of other keys is the value of the branch where it
 * ends (the branch's 17th item, Node.scala:31-40).  nseg tries as in
 * kh_trie_roots_segmented (koff / voff indexed like the inputs).  The generic key path
 * of MerklePatriciaTrie.put with an identity key serializer (trie/package.scala:28-36). */
int kh_trie_roots_varkeys(const uint8_t* keys, const uint64_t* koff, const uint8_t* vals, const uint64_t* voff,
                          const uint64_t* seg_off, uint64_t nseg, uint8_t* roots32, kh_stats* stats);

/* List tries (transactions / receipts / ommers roots): item i of trie s, i.e. input
 * seg_off[s] + i, is put under key rlp(i) (MptListValidator.isValid,
 * khipu-eth/.../validators/MptListValidator.scala:15-46; BlockGenerator.scala:157-163);
 * items[off[j] .. off[j+1]) is the serialized item.  Keys are made on the device. */
int kh_list_roots(const uint8_t* items, const uint64_t* off, const uint64_t* seg_off, uint64_t nseg,
                  uint8_t* roots32, kh_stats* stats);

/* kh_trie_roots_segmented over ngpus GPUs of this process (SURVEY §8e, configs[3]): the
 * tries are split into contiguous ranges of about equal slot counts, one per device (a
 * device may repeat), each built as one segmented build; roots32 receives every trie's
 * root in order.  The tries are independent: no data moves between the GPUs. */
int kh_trie_roots_segmented_sharded(const int* devices, int ngpus, const uint8_t* keys, uint32_t klen,
                                    const uint8_t* vals, const uint64_t* voff, const uint64_t* seg_off, uint64_t nseg,
                                    uint32_t flags, uint8_t* roots32, kh_stats* stats);

/* The kh_trie_root result computed on ngpus GPUs of this process: the
 * puts are split into ngpus contiguous slices, slice g staged to devices[g], keys hashed
 * there, records routed to the owner of their top key nibble (q * ngpus >> 4) over RCCL
 * point-to-point (xGMI), every owner builds its subtries from nibble 1, and the 16
 * references are folded into the root branch.  Devices must be distinct for the RCCL
 * exchange; a list that repeats a device runs several shards on it (device copies).
 * The keys are exchanged first; the value lengths and bytes follow on a stream of their
 * own while every owner sorts its keys and derives the topology.
 * stats: sums over the shards; t_keys_ms / t_sort_ms / t_total_ms are the host wall
 * times of stage+hash+partition / key exchange / the whole call.  Host buffers. */
int kh_trie_root_sharded(const int* devices, int ngpus, const uint8_t* keys, uint32_t klen, const uint8_t* vals,
                         const uint64_t* voff, uint64_t n, uint32_t flags, uint8_t root32[32], kh_stats* stats);

/* kh_list_roots with the items in HBM: d_off holds the offsets of every item of the call
 * into d_items (item j at d_items[d_off[j] .. d_off[j+1]), j from h_seg_off[0]); the
 * segment offsets are host memory. */
int kh_dev_list_roots(kh_ctx* ctx, const uint8_t* d_items, const uint64_t* d_off, const uint64_t* h_seg_off,
                      uint64_t nseg, uint8_t* roots32, kh_stats* stats);

/* Root plus every node a fresh node store needs: each node reachable from the root
 * whose encoding is >= 32 B, plus the root node (MerklePatriciaTrie.scala:505-511).
 * Node j: hash hashes32[32j..), encoding rlp[off[j] .. off[j+1]) (off has n_nodes+1
 * entries).  Nodes are ordered leaves first, then branches/extensions bottom-up, the
 * root last.  On KH_ENOSPC, *n_nodes and *rlp_len report the sizes needed. */
int kh_trie_root_nodes(const uint8_t* keys, uint32_t klen, const uint8_t* vals, const uint64_t* voff, uint64_t n,
                       uint32_t flags, uint8_t root32[32], uint8_t* hashes32, uint64_t node_cap, uint8_t* rlp,
                       uint64_t rlp_cap, uint64_t* off, uint64_t* n_nodes, uint64_t* rlp_len, kh_stats* stats);

/* ---- device-resident interface (inputs already in HBM; used by bench.py and the
 *      multi-GPU driver).  One context per device; a context is not shared across
 *      threads without external synchronisation. ---- */

int kh_ctx_create(int device, kh_ctx** out);
int kh_ctx_destroy(kh_ctx* ctx);
/* Use an existing HIP stream (hipStream_t passed as void*); NULL = the context's own stream. */
int kh_ctx_set_stream(kh_ctx* ctx, void* hip_stream);

int kh_dev_kec256_batch(kh_ctx* ctx, const uint8_t* d_data, const uint64_t* d_off, uint64_t n, uint8_t* d_out32);

/* Build over device inputs.  depth0 = 0: one trie (or one per segment when d_seg is
 * non-NULL: d_seg[i] = segment id of input i, ids < nseg).  depth0 = 1, d_seg NULL:
 * the 16 top-nibble subtries of one trie, paths starting at nibble 1 (the shard
 * unit of the multi-GPU path).  Per result r (nseg or 16 of them):
 *   h_hash32[32r..)  kec256 of the top node's encoding (the root for depth0 = 0);
 *   h_enc_len[r]     that encoding's length (0 = empty);
 *   h_inline32[32r..) the encoding itself when shorter than 32 B (capped reference).
 * Outputs are host buffers; h_inline32 may be NULL. */
int kh_dev_trie_build(kh_ctx* ctx, const uint8_t* d_keys, uint32_t klen, const uint8_t* d_vals,
                      const uint64_t* d_voff, uint64_t n, const uint32_t* d_seg, uint64_t nseg, uint32_t depth0,
                      uint32_t flags, uint8_t* h_hash32, uint32_t* h_enc_len, uint8_t* h_inline32,
                      kh_stats* stats);

/* kh_dev_trie_build whose values arrive later (the multi-GPU exchange): the keys must be
 * in place when it is called; d_vals / d_voff are read only after the HIP event
 * vals_ready (a hipEvent_t recorded on any stream of the context's device; NULL = ready)
 * has completed, so the key sort and the branch topology run while the values are
 * still in flight. */
int kh_dev_trie_build_ev(kh_ctx* ctx, void* vals_ready, const uint8_t* d_keys, uint32_t klen,
                         const uint8_t* d_vals, const uint64_t* d_voff, uint64_t n, const uint32_t* d_seg,
                         uint64_t nseg, uint32_t depth0, uint32_t flags, uint8_t* h_hash32, uint32_t* h_enc_len,
                         uint8_t* h_inline32, kh_stats* stats);

/* Fold 16 capped top-nibble references (as produced by kh_dev_trie_build with depth0 = 1,
 * gathered from every shard) into the root: kec256(RLP[ref_0..ref_15, ""]).
 * Requires >= 2 non-empty references (otherwise the root is not a branch: returns KH_EINVAL
 * and the caller builds on one device). */
int kh_fold_root16(const uint8_t* hash32x16, const uint32_t* enc_len16, const uint8_t* inline32x16,
                   uint8_t root32[32]);

/* kec256 of n keys of klen bytes (device buffers; the KH_HASH_KEYS step on its own). */
int kh_dev_hash_keys(kh_ctx* ctx, const uint8_t* d_keys, uint32_t klen, uint64_t n, uint8_t* d_out32);

/* Multi-GPU routing: stable partition of n records (32-byte trie keys + packed values) by
 * owner = top nibble * nparts / 16 (nparts <= 16).  Writes the records grouped by owner
 * (input order kept inside a group, so later puts still win after the exchange):
 * d_out_keys (n*32 B), d_out_vals (total value bytes), d_out_vlen (n value lengths);
 * h_counts[p] / h_bytes[p] = records / value bytes for owner p (host).  d_keys32, d_voff,
 * d_out_keys, d_out_vals and d_out_vlen must be 8-byte aligned (KH_EINVAL otherwise). */
int kh_dev_partition(kh_ctx* ctx, const uint8_t* d_keys32, const uint8_t* d_vals, const uint64_t* d_voff,
                     uint64_t n, uint32_t nparts, uint8_t* d_out_keys, uint8_t* d_out_vals, uint64_t* d_out_vlen,
                     uint64_t* h_counts, uint64_t* h_bytes);
/* The same with the value copy deferred: it returns once the keys, the lengths, the counts
 * and the bytes per owner are in place, the value bytes still being copied on the context's stream;
 * vals_done (a hipEvent_t of the context's device) is recorded after them.  NULL
 * vals_done: kh_dev_partition. */
int kh_dev_partition_ev(kh_ctx* ctx, void* vals_done, const uint8_t* d_keys32, const uint8_t* d_vals,
                        const uint64_t* d_voff, uint64_t n, uint32_t nparts, uint8_t* d_out_keys,
                        uint8_t* d_out_vals, uint64_t* d_out_vlen, uint64_t* h_counts, uint64_t* h_bytes);
/* kh_dev_hash_keys and kh_dev_partition_ev in one call: the n klen-byte keys (addresses)
 * are kec256'd in a pass that also writes each key's owner as a byte, so the count pass
 * reads those bytes instead of the hashed keys (what the sharded step runs at N > 1).  Same outputs as kh_dev_partition_ev over
 * kh_dev_hash_keys(d_keys) (the hashed keys are written only to d_out_keys, grouped). */
int kh_dev_hash_partition_ev(kh_ctx* ctx, void* vals_done, const uint8_t* d_keys, uint32_t klen,
                             const uint8_t* d_vals, const uint64_t* d_voff, uint64_t n, uint32_t nparts,
                             uint8_t* d_out_keys, uint8_t* d_out_vals, uint64_t* d_out_vlen, uint64_t* h_counts,
                             uint64_t* h_bytes);

/* ---- fast-sync NodeData verification ----
 * NodeDatasRequest.processResponse (sync/package.scala:81-125) over a batch of peer
 * values: kec256 each value (data packed, off[n+1]), match it against the nreq
 * requested hashes (req32, req_kind[r]: 0 state trie node, 1 storage root, 2 contract
 * storage node, 3 EVM code; a duplicate hash takes the last request's kind), and
 * decode a matched trie node with PV63's MptNode rules (PV63.scala:96-127) to list the
 * children still to fetch: getStateNodeChildren / getContractMptNodeChildren
 * (sync/package.scala:127-165) — branch / extension child hashes, and for a state
 * leaf the account's codeHash (kind 3) then stateRoot (kind 1) unless empty.
 * Per value i (host buffers; any output may be NULL):
 *   hash32[32i..)          kec256(value)
 *   match[i]               matched request index, -1 if none (then nothing is decoded)
 *   status[i]              0 ok, 1 not a trie node ("Cannot decode NodeData"),
 *                          2 bad child ("unexpected value in node"), 3 bad account
 *                          ("Cannot decode Account"), 4 malformed RLP
 *   nchild[i], child32[512i..), child_kind[16i..)   children in the reference's order */
int kh_verify_nodes(const uint8_t* data, const uint64_t* off, uint64_t n, const uint8_t* req32, const uint8_t* req_kind,
                    uint64_t nreq, uint8_t* hash32, int64_t* match, uint8_t* status, uint8_t* nchild, uint8_t* child32,
                    uint8_t* child_kind);
/* The same with the children packed, as processResponse concatenates them (childHashes :::
 * hashes): value i's children are child32[32k..) / child_kind[k] for k in
 * [child_off[i], child_off[i+1]) (child_off has n+1 entries); *n_children = the total.  When
 * the total exceeds child_cap (16 n always suffices) the call returns KH_ENOSPC after writing
 * every other output, child_off and *n_children. */
int kh_verify_nodes_packed(const uint8_t* data, const uint64_t* off, uint64_t n, const uint8_t* req32,
                           const uint8_t* req_kind, uint64_t nreq, uint8_t* hash32, int64_t* match, uint8_t* status,
                           uint64_t* child_off, uint8_t* child32, uint8_t* child_kind, uint64_t child_cap,
                           uint64_t* n_children);

/* ---- resident tries and forests: incremental commit ----
 * A trie kept in HBM between commits as node records found by their anchor (trie id,
 * depth, key prefix): khipu_amd/csrc/forest.h.  Replaces the per-key fold of
 * TrieAccounts.flush / TrieStorage.flush (TrieAccounts.scala:22-28, TrieStorage.scala:43-60)
 * over MerklePatriciaTrie.put / remove (MerklePatriciaTrie.scala:157-281, 290-477): a commit
 * opens only the nodes on the changed keys' paths and rebuilds them (with the canonical
 * `fix` collapse of :430-477), O(dirty keys x depth) work.  A FOREST holds many tries
 * (contract storage tries, BlockWorldState.scala:243-252) in one handle, each op tagged
 * with its trie id; one commit re-roots every trie the block touched.  Device-buffer
 * entry points use the handle's context stream (one thread at a time per handle); the
 * _host variants take host buffers (what the JNI shim binds).
 * Semantics of a commit: nup upserts then ndel deletes, the last op on a key winning;
 * deleting an absent key is a no-op; keys are klen bytes (32, or any with KH_HASH_KEYS,
 * which must match the flag the trie was opened with). */
typedef struct kh_trie kh_trie;

/* Open a trie from n records (duplicates: the later wins).  flags: KH_HASH_KEYS, KH_EMIT_NODES. */
int kh_trie_open(kh_ctx* ctx, const uint8_t* d_keys, uint32_t klen, const uint8_t* d_vals, const uint64_t* d_voff,
                 uint64_t n, uint32_t flags, uint8_t root32[32], kh_trie** out);
int kh_trie_open_host(const uint8_t* keys, uint32_t klen, const uint8_t* vals, const uint64_t* voff, uint64_t n,
                      uint32_t flags, uint8_t root32[32], kh_trie** out);

/* Open a trie from its root hash and a node store: MerklePatriciaTrie.apply(
 * rootHash, source) with getNode (MerklePatriciaTrie.scala:60-66,520-542).  The store holds
 * n node encodings enc[off[i] .. off[i+1]), keyed by their kec256 (content addressed, as
 * NodeStorage is); the nodes reachable from root32 are decoded on the device.  A node
 * missing from the store returns KH_ENODE with its hash in missing32
 * (MPTNodeMissingException); EMPTY_TRIE_HASH opens an empty trie. */
int kh_trie_open_nodes(kh_ctx* ctx, const uint8_t root32[32], const uint8_t* d_enc, const uint64_t* d_off, uint64_t n,
                       uint32_t flags, uint8_t missing32[32], kh_trie** out);
int kh_trie_open_nodes_host(const uint8_t root32[32], const uint8_t* enc, const uint64_t* off, uint64_t n,
                            uint32_t flags, uint8_t missing32[32], kh_trie** out);

/* One commit; root32 receives the new root.  stats: n_node_hashes counts the nodes re-hashed.
 * A handle without KH_EMIT_NODES returns once the new roots are on the host: the commit's
 * record and anchor-map writes finish on the library's stream after it (every later call on
 * the handle is ordered after them; an internal failure there surfaces at the next call). */
int kh_trie_apply(kh_trie* h, const uint8_t* d_up_keys, const uint8_t* d_up_vals, const uint64_t* d_up_voff,
                  uint64_t nup, const uint8_t* d_del_keys, uint64_t ndel, uint32_t klen, uint32_t flags,
                  uint8_t root32[32], kh_stats* stats);
int kh_trie_apply_host(kh_trie* h, const uint8_t* up_keys, const uint8_t* up_vals, const uint64_t* up_voff,
                       uint64_t nup, const uint8_t* del_keys, uint64_t ndel, uint32_t klen, uint32_t flags,
                       uint8_t root32[32], kh_stats* stats);

/* A forest of tries (empty).  ctx NULL: the shared context of the current device, the one
 * the *_host entry points use (so kh_block_commit_host can pair it with a trie opened by
 * kh_trie_open_host).  Each op names its trie (any uint32 id).  After a commit,
 * h_tries / h_roots32 receive the touched tries (ascending ids) and their new roots
 * (EMPTY_TRIE_HASH for a trie left empty); KH_ENOSPC with *n_tries when cap is short. */
int kh_forest_open(kh_ctx* ctx, uint32_t flags, kh_trie** out);
int kh_forest_apply(kh_trie* f, const uint32_t* d_up_trie, const uint8_t* d_up_keys, const uint8_t* d_up_vals,
                    const uint64_t* d_up_voff, uint64_t nup, const uint32_t* d_del_trie, const uint8_t* d_del_keys,
                    uint64_t ndel, uint32_t klen, uint32_t* h_tries, uint8_t* h_roots32, uint64_t cap,
                    uint64_t* n_tries, kh_stats* stats);
int kh_forest_apply_host(kh_trie* f, const uint32_t* up_trie, const uint8_t* up_keys, const uint8_t* up_vals,
                         const uint64_t* up_voff, uint64_t nup, const uint32_t* del_trie, const uint8_t* del_keys,
                         uint64_t ndel, uint32_t klen, uint32_t* h_tries, uint8_t* h_roots32, uint64_t cap,
                         uint64_t* n_tries, kh_stats* stats);

/* The touched tries and roots of a forest's last commit (also after kh_block_commit). */
int kh_forest_last_roots(kh_trie* f, uint32_t* h_tries, uint8_t* h_roots32, uint64_t cap, uint64_t* n_tries);

/* One block (BlockWorldState.flush, BlockWorldState.scala:243-252 then TrieAccounts.flush):
 * the storage ops into the forest, each touched trie's new root written into the stateRoot
 * field of the account upserts that name it (d_a_up_trie[i], KH_NO_TRIE for none; the body
 * RLP[nonce, balance, stateRoot, codeHash] of PV63.scala:46-51 is patched in place in
 * d_a_up_vals), then the account ops into the state trie.  One call per block. */
int kh_block_commit(kh_trie* state, kh_trie* storage, const uint32_t* d_s_up_trie, const uint8_t* d_s_up_keys,
                    const uint8_t* d_s_up_vals, const uint64_t* d_s_up_voff, uint64_t ns_up,
                    const uint32_t* d_s_del_trie, const uint8_t* d_s_del_keys, uint64_t ns_del, uint32_t s_klen,
                    const uint8_t* d_a_up_keys, uint8_t* d_a_up_vals, const uint64_t* d_a_up_voff,
                    const uint32_t* d_a_up_trie, uint64_t na_up, const uint8_t* d_a_del_keys, uint64_t na_del,
                    uint32_t a_klen, uint8_t state_root32[32], kh_stats* stats);
/* kh_block_commit from host arrays (staged in one device buffer; for a JVM caller). */
int kh_block_commit_host(kh_trie* state, kh_trie* storage, const uint32_t* s_up_trie, const uint8_t* s_up_keys,
                         const uint8_t* s_up_vals, const uint64_t* s_up_voff, uint64_t ns_up,
                         const uint32_t* s_del_trie, const uint8_t* s_del_keys, uint64_t ns_del, uint32_t s_klen,
                         const uint8_t* a_up_keys, const uint8_t* a_up_vals, const uint64_t* a_up_voff,
                         const uint32_t* a_up_trie, uint64_t na_up, const uint8_t* a_del_keys, uint64_t na_del,
                         uint32_t a_klen, uint8_t state_root32[32], kh_stats* stats);

/* ---- versioned commits ----
 * Ledger.executeBlock flushes the parallel attempt's world state and, when its root does not
 * validate, re-executes the block sequentially from the SAME parent state
 * (khipu-eth/.../ledger/Ledger.scala:237-271); validateBlockAfterExecution rejects a block whose
 * root or gas does not match (:603-620); TrieAccounts.rootHash flushes a COPY of the trie and
 * leaves the trie itself untouched (khipu-eth/.../ledger/TrieAccounts.scala:73-80, called per
 * transaction at Ledger.scala:576; MerklePatriciaTrie.copy, MerklePatriciaTrie.scala:556).
 *
 * kh_trie_savepoint opens a savepoint on a trie or forest (they nest; *depth = the number now
 * open).  Commits after it are journaled: each saves the records it rewrites and logs the
 * anchor-map slots it changes, O(changed nodes).  kh_trie_rollback returns the handle to the
 * innermost savepoint's version -- root, records, value heap, the last commit's trie list and
 * roots (kh_forest_last_roots) and write-back set (kh_trie_emit_nodes) -- and closes it;
 * kh_trie_release keeps the commits and closes it.  kh_block_commit is all or nothing on both
 * handles: a refusal or failure in either phase leaves both at the parent version. */
int kh_trie_savepoint(kh_trie* h, uint32_t* depth);
int kh_trie_rollback(kh_trie* h);
int kh_trie_release(kh_trie* h);
int kh_trie_savepoint_depth(const kh_trie* h, uint32_t* depth);

/* TrieAccounts.rootHash (TrieAccounts.scala:73-80): the root that kh_trie_apply of this batch
 * would give, the handle left unchanged (a commit between a savepoint and its rollback). */
int kh_trie_root_of(kh_trie* h, const uint8_t* d_up_keys, const uint8_t* d_up_vals, const uint64_t* d_up_voff,
                    uint64_t nup, const uint8_t* d_del_keys, uint64_t ndel, uint32_t klen, uint32_t flags,
                    uint8_t root32[32], kh_stats* stats);
int kh_trie_root_of_host(kh_trie* h, const uint8_t* up_keys, const uint8_t* up_vals, const uint64_t* up_voff,
                         uint64_t nup, const uint8_t* del_keys, uint64_t ndel, uint32_t klen, uint32_t flags,
                         uint8_t root32[32], kh_stats* stats);

/* MerklePatriciaTrie.copy (MerklePatriciaTrie.scala:556): an independent handle holding the
 * current version of h in HBM (no savepoints); free it with kh_trie_free. */
int kh_trie_copy(kh_trie* h, kh_trie** out);

/* Storage write-back hand-off of the LAST commit (open or apply) of a
 * trie opened with KH_EMIT_NODES: exactly the nodes that commit created -- every node
 * reachable from a new root whose encoding is >= 32 B and that the previous version did
 * not hold, plus a changed root node -- what persist()/changes hand to NodeStorage.update
 * (MerklePatriciaTrie.scala:491-516,544-554; BlockWorldState.scala:312-330).  Same layout
 * and KH_ENOSPC size negotiation as kh_trie_root_nodes (no re-encoding on the retry). */
int kh_trie_emit_nodes(kh_trie* h, uint8_t* hashes32, uint64_t node_cap, uint8_t* rlp, uint64_t rlp_cap,
                       uint64_t* off, uint64_t* n_nodes, uint64_t* rlp_len);

/* Batched get on a resident trie or forest: MerklePatriciaTrie.get (MerklePatriciaTrie.scala:
 * 90-147; callers Blockchain.scala:336-342) answered from the records in HBM by the commit's
 * anchor descent, so a JVM holding state in HBM can read it without its own node store.
 * n queries: key i (klen bytes; kec256'd on the device when the trie was opened with
 * KH_HASH_KEYS, as its commits are) in trie trie[i] (forests; NULL for a single trie).
 * found[i] = 1 iff the key is present (None otherwise); the values are packed into vals with
 * voff[n+1] (an absent key has an empty span).  When the values need more than val_cap
 * bytes the call returns KH_ENOSPC and writes only *val_bytes (the size needed).
 * Device-buffer form on the handle's context stream; _host form with host buffers. */
int kh_trie_get(kh_trie* h, const uint32_t* d_trie, const uint8_t* d_keys, uint32_t klen, uint64_t n,
                uint8_t* d_vals, uint64_t val_cap, uint64_t* d_voff, uint8_t* d_found, uint64_t* val_bytes);
int kh_trie_get_host(kh_trie* h, const uint32_t* trie, const uint8_t* keys, uint32_t klen, uint64_t n,
                     uint8_t* vals, uint64_t val_cap, uint64_t* voff, uint8_t* found, uint64_t* val_bytes);

/* Leaves of a trie (of all tries of a forest). */
/* HBM held by a resident trie or forest.  Records and the value heap are append-only between
 * compactions: a commit appends the records and values it makes and leaves the ones it
 * replaces dead (~18 MB per configs[2] block).  records / heap_bytes: in use; live_records /
 * live_heap_bytes: the current version's (counted on the device); map_slots: anchor-map
 * capacity; hbm_bytes: every buffer the handle holds. */
typedef struct kh_trie_usage_t {
  uint64_t records, live_records, heap_bytes, live_heap_bytes, map_slots, hbm_bytes;
} kh_trie_usage_t;
int kh_trie_usage(kh_trie* h, kh_trie_usage_t* u);
/* Rewrite the live records and their values densely and rebuild the anchor map (O(records)
 * on the device; the version -- roots, last roots, write-back set -- is unchanged).  The JVM
 * calls it between blocks when dead records pass a budget.  KH_EINVAL while a savepoint is
 * open (the journal holds record indices).  before (nullable): records / heap bytes before. */
int kh_trie_compact(kh_trie* h, kh_trie_usage_t* before);
int kh_trie_size(const kh_trie* h, uint64_t* n);
int kh_trie_free(kh_trie* h);

/* Synthetic account generator (pinned in khipu_amd/csrc/synth.h): writes
 * accounts [first, first+n) of config `cfg` — 20-byte addresses (d_addr, n*20 B) and RLP
 * account bodies packed at d_vals with d_voff[n+1] (offsets relative to d_vals; d_vals
 * must hold n*96 B).  Deterministic; the CPU restatement lives in tests. */
int kh_dev_synth_accounts(kh_ctx* ctx, uint32_t cfg, uint64_t first, uint64_t n, uint8_t* d_addr,
                          uint8_t* d_vals, uint64_t* d_voff);

/* Synthetic contract storage tries [t0, t0+nt) of config cfg (pinned in
 * khipu_amd/csrc/synth.h: log-uniform 1..10^4 slots per trie, 32-byte big-endian slot
 * words as keys -- hash them with KH_HASH_KEYS -- and RLP(trimmed 1-32 byte) values).
 * Always: d_seg_off[nt+1] (each trie's first slot, from 0), *n_slots, *val_bytes.  With
 * d_keys non-NULL also the slots: keys (n_slots*32 B), packed values (d_vals, val_bytes B)
 * with d_voff[n_slots+1], and d_seg[n_slots] = trie - t0 (the segment ids of
 * kh_dev_trie_build).  Deterministic per trie: any range can be made on any GPU. */
int kh_dev_synth_storage(kh_ctx* ctx, uint32_t cfg, uint64_t t0, uint64_t nt, uint64_t* d_seg_off, uint64_t* n_slots,
                         uint64_t* val_bytes, uint8_t* d_keys, uint8_t* d_vals, uint64_t* d_voff, uint32_t* d_seg);

#ifdef __cplusplus
}
#endif
#endif /* KHST_H */
