/*
 * huffgpu.h — C ABI of the MI355X-native Huffman byte codec.
 *
 * This is the drop-in boundary for the hot path of k-xlsx/huff-encoding
 * (reference read-only at /root/reference; citations are file:line there).
 * The reference is Rust; a Rust host would bind these functions with
 * `extern "C"` declarations (see INTEGRATION.md for the binding stub).
 *
 * Conventions
 *  - Every function returns an int status (HUFF_OK == 0). No exception or
 *    panic crosses the ABI: every reference panic becomes a distinct status,
 *    and huff_last_error() returns the reference's message (thread-local).
 *  - Plain pointers and sizes only. "host" pointers are CPU memory; "d_"
 *    pointers are device (HBM) memory of the context's GPU.
 *  - One huff_ctx per host thread. A context owns its HIP stream (or adopts
 *    the caller's via huff_ctx_set_stream) and its device workspace. The own
 *    stream is a blocking stream, so it runs after work already queued on the
 *    legacy default stream (PyTorch's default). Calls on
 *    different contexts are thread-safe; the host-only functions (weights,
 *    tree) are reentrant and need no context.
 *  - This header is the u8 alphabet (the reference's ByteWeights path); the
 *    other integer letter types are in huffgpu_wide.h.
 */
#ifndef HUFFGPU_H
#define HUFFGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------ */
/* status codes                                                              */
/* ------------------------------------------------------------------------ */
enum huff_status {
    HUFF_OK = 0,
    HUFF_E_INVALID_ARG = 1,     /* NULL / out-of-range argument                          */
    HUFF_E_EMPTY_WEIGHTS = 2,   /* panic "provided empty weights" tree_inner.rs:283-285  */
    HUFF_E_MISSING_LETTER = 3,  /* CompressError "letter not found in codes" comp.rs:426  */
    HUFF_E_FROM_BIN = 4,        /* FromBinError tree_inner.rs:530-590                     */
    HUFF_E_FROM_BYTES = 5,      /* CompressedDataFromBytesError comp.rs:128-184           */
    HUFF_E_BUFFER_TOO_SMALL = 6,/* caller buffer too small; *_len outputs hold the need   */
    HUFF_E_CODE_TOO_LONG = 7,   /* a code too long for the requested view (u64 code table, */
                                /* wide letters' kernels); byte-path compress/decompress  */
                                /* take any length (deep.hip)                             */
    HUFF_E_HIP = 8,             /* HIP runtime error (message has the HIP error string)   */
    HUFF_E_IO = 9,              /* ErrorKind::Io huff/src/error.rs                         */
    HUFF_E_UNRECOGNIZED = 10,   /* ErrorKind::UnrecognizedFormat                           */
    HUFF_E_MISSING_HEADER = 11, /* ErrorKind::MissingHeaderInfo huff/src/comp.rs:95-128   */
    HUFF_E_INVALID_HEADER = 12, /* ErrorKind::InvalidHeaderInfo huff/src/comp.rs:107-144  */
    HUFF_E_TIMEOUT = 13,        /* a bounded device wait expired (never expected)         */
    HUFF_E_EMPTY_COMP = 14,     /* panic "provided comp_bytes are empty" comp.rs:56-58    */
    HUFF_E_PADDING = 15,        /* panic "padding bits cannot be larger than 7" comp.rs:59 */
    HUFF_E_TREE_LEN = 16,       /* panic "stored tree length must be at least 2" :153-155 */
    HUFF_E_NO_DEVICE = 17,      /* no GPU / HIP unavailable: the product never falls back */
    HUFF_E_STATE = 18,          /* call order violated (e.g. pack before hist), or a decode
                                 * tree whose codes differ from the packed tree's          */
    HUFF_E_CORRUPT = 19         /* decode self-check (HUFF_DEC_VARIANT 11-13) found a lane
                                 * that did not end at its successor's restart point        */
};

/* Message of the last failing call on this thread (reference wording). */
const char* huff_last_error(void);
/* The letter of the last HUFF_E_MISSING_LETTER (CompressError::missing_letter, comp.rs:587). */
uint8_t huff_last_missing_letter(void);
const char* huff_version(void);

/* ------------------------------------------------------------------------ */
/* context                                                                    */
/* ------------------------------------------------------------------------ */
typedef struct huff_ctx huff_ctx;

int huff_ctx_create(int device, huff_ctx** out);
int huff_ctx_destroy(huff_ctx* ctx);
/* Adopt a caller stream (hipStream_t); NULL reverts to the context's own. */
int huff_ctx_set_stream(huff_ctx* ctx, void* hip_stream);
int huff_ctx_synchronize(huff_ctx* ctx);
int huff_ctx_device(const huff_ctx* ctx);
/* Kernel timing (tracing aux subsystem): when on, every kernel the context
 * launches is bracketed by HIP events on the context's stream. */
int huff_ctx_set_timing(huff_ctx* ctx, int on);
/* Sum of the timed durations (ms) and launch count of kernel `name`
 * ("hist", "chunk_bits", "scan", "pack", "decode", "indexless_*") since the
 * last reset; synchronises the stream. */
int huff_ctx_kernel_time(huff_ctx* ctx, const char* name, double* total_ms, uint64_t* launches);
int huff_ctx_reset_timing(huff_ctx* ctx);

/* ------------------------------------------------------------------------ */
/* ByteWeights — huff_coding/src/weights.rs:174-443                          */
/* ------------------------------------------------------------------------ */
typedef struct {
    uint64_t weights[256];   /* weights.rs:176 */
    uint64_t len;            /* weights.rs:177 number of distinct bytes */
} huff_byte_weights;

/* ByteWeights::new (weights.rs:245-250) */
void huff_weights_new(huff_byte_weights* out);
/* ByteWeights::from_bytes (weights.rs:265-279), counted by the hist256 kernel.
 * `bytes` is host memory. */
int huff_weights_from_bytes(huff_ctx* ctx, const uint8_t* bytes, size_t n, huff_byte_weights* out);
/* ByteWeights::threaded_from_bytes (weights.rs:293-319 + utils.rs:6-28): one
 * GPU histogram per ration, merged with the reference's merge order/quirk. */
int huff_weights_threaded_from_bytes(huff_ctx* ctx, const uint8_t* bytes, size_t n,
                                     size_t thread_num, huff_byte_weights* out);
/* add_byte_weights / AddAssign (weights.rs:222-235,374-387), quirk included. */
void huff_weights_add(huff_byte_weights* self, const huff_byte_weights* other);
/* Iter::next order (weights.rs:423-441), wrap duplicate included; returns the
 * number of (letter, weight) pairs written (<= 257). */
size_t huff_weights_iter(const huff_byte_weights* w, uint8_t letters[257], uint64_t weights[257]);

/* ------------------------------------------------------------------------ */
/* HuffTree — huff_coding/src/tree/tree_inner.rs                             */
/* ------------------------------------------------------------------------ */
typedef struct huff_tree huff_tree;

/* HuffTree::from_weights (tree_inner.rs:281-320) with the reference's exact
 * BinaryHeap tie order (branch_heap.rs:18-83). HUFF_E_EMPTY_WEIGHTS on empty. */
int huff_tree_from_weights(const huff_byte_weights* w, huff_tree** out);
int huff_tree_clone(const huff_tree* t, huff_tree** out);
void huff_tree_free(huff_tree* t);
size_t huff_tree_num_leaves(const huff_tree* t);
uint64_t huff_tree_root_weight(const huff_tree* t);
/* read_codes (tree_inner.rs:356-419): right-aligned code and bit length per
 * byte, len 0 = no code. HUFF_E_CODE_TOO_LONG if a code exceeds 64 bits (use
 * huff_tree_code_bits then). */
int huff_tree_read_codes(const huff_tree* t, uint64_t code[256], uint8_t len[256]);
/* one code as a bit string (one bit per byte), any length */
int huff_tree_code_bits(const huff_tree* t, uint8_t letter, uint8_t* bits, size_t cap, size_t* nbits);
/* as_bin (tree_inner.rs:632-668): packed Msb0 bytes with zero tail bits. */
int huff_tree_as_bin(const huff_tree* t, uint8_t* out, size_t cap, size_t* nbits);
/* try_from_bin (tree_inner.rs:522-604): `bits` packed Msb0, nbits used. */
int huff_tree_try_from_bin(const uint8_t* bits, size_t nbits, huff_tree** out);

/* Walking the tree: the reference's HuffTree::root (tree_inner.rs:322-325)
 * and HuffBranch / HuffLeaf accessors. A branch is a node id (>= 0) valid as
 * long as the tree; -1 stands for None. HUFF_E_INVALID_ARG for a null tree or
 * an id the tree does not hold. */
int huff_tree_root(const huff_tree* t, int32_t* branch);
/* HuffBranch::left_child / right_child (branch.rs:254-268): both -1 when the
 * branch has no children (has_children, branch.rs:277-279; children_iter
 * returns None then, else left then right, branch.rs:247-250). */
int huff_branch_children(const huff_tree* t, int32_t branch, int32_t* left, int32_t* right);
/* HuffBranch::leaf (branch.rs:207-209) -> HuffLeaf::letter / weight
 * (leaf.rs:61-68): *has_letter = 1 and *letter for a letter branch, 0 for a
 * joint branch (letter None). Weights are 0 in a tree read by try_from_bin
 * (tree_inner.rs:446-447). Any output pointer may be NULL. */
int huff_branch_leaf(const huff_tree* t, int32_t branch, int* has_letter, uint8_t* letter, uint64_t* weight);
/* HuffLeaf::code (leaf.rs:70-73): the branch's path from the root, one bit
 * per byte (tree_inner.rs:422-440 sets it on every branch below the root; a
 * single-leaf root gets [0], tree_inner.rs:310-315). *has_code = 0 (None) for
 * the root of a tree with children. HUFF_E_BUFFER_TOO_SMALL if cap < *nbits. */
int huff_branch_code(const huff_tree* t, int32_t branch, uint8_t* bits, size_t cap, size_t* nbits, int* has_code);

/* ------------------------------------------------------------------------ */
/* CompressData + compress/decompress — huff_coding/src/comp.rs              */
/* ------------------------------------------------------------------------ */
typedef struct huff_compress_data huff_compress_data;

/* CompressData::new (comp.rs:55-68): HUFF_E_EMPTY_COMP / HUFF_E_PADDING. */
int huff_cd_new(const uint8_t* comp, size_t len, uint8_t padding, const huff_tree* t,
                huff_compress_data** out);
void huff_cd_free(huff_compress_data* cd);
int huff_cd_comp_bytes(const huff_compress_data* cd, const uint8_t** ptr, size_t* len);
uint8_t huff_cd_padding(const huff_compress_data* cd);
const huff_tree* huff_cd_tree(const huff_compress_data* cd);
/* whether the GPU restart index of the encoder is attached (decode fast path) */
int huff_cd_has_index(const huff_compress_data* cd);
/* CompressData::to_bytes (comp.rs:279-300) */
int huff_cd_to_bytes(const huff_compress_data* cd, uint8_t* out, size_t cap, size_t* out_len);
/* CompressData::try_from_bytes (comp.rs:128-184) */
int huff_cd_try_from_bytes(const uint8_t* bytes, size_t n, huff_compress_data** out);

/* compress_with_tree (comp.rs:419-451) on the GPU; the tree is borrowed (the
 * reference consumes it and hands it back in CompressData; here it is cloned).
 * `bytes` is host memory. */
int huff_compress_with_tree(huff_ctx* ctx, const uint8_t* bytes, size_t n, const huff_tree* t,
                            huff_compress_data** out);
/* ByteWeights::from_bytes + HuffTree::from_weights + compress_with_tree: the
 * deterministic byte path (comp.rs:353-356 `compress` uses a RandomState
 * HashMap and is not reproducible under ties). */
int huff_compress_bytes(huff_ctx* ctx, const uint8_t* bytes, size_t n, huff_compress_data** out);
/* decompress (comp.rs:487-519) on the GPU. out_len receives the symbol count;
 * if cap is too small, HUFF_E_BUFFER_TOO_SMALL and *out_len = needed. */
int huff_decompress(huff_ctx* ctx, const huff_compress_data* cd, uint8_t* out, size_t cap,
                    size_t* out_len);

/* ------------------------------------------------------------------------ */
/* device-resident encode job (benchmarks, multi-GPU shards)                 */
/* ------------------------------------------------------------------------ */
typedef struct huff_enc huff_enc;

/* An encode job over n bytes already resident in HBM (d_in 16-B aligned). */
int huff_enc_create(huff_ctx* ctx, const uint8_t* d_in, size_t n, huff_enc** out);
void huff_enc_free(huff_enc* e);
/* pass 1: hist256 over the job (per-chunk + global); weights to host */
int huff_enc_hist(huff_enc* e, uint64_t weights[256]);
/* pass 1 queued ahead, without waiting for it: the next huff_enc_hist or
 * huff_enc_compress of this job only waits for its weights. Queued between a
 * job's pack and its decode, the next job's host tree build overlaps that
 * decode (a streaming encoder's software pipeline; no reference counterpart).
 * One pending pass 1 per context: another job's hist/compress/hist_launch on
 * the same context fails with HUFF_E_STATE until this job's is waited for. */
int huff_enc_hist_launch(huff_enc* e);
/* pass 1 for a sharded job without a host round trip (replaces
 * the per-shard ByteWeights::threaded_from_bytes + merge, weights.rs:293-319):
 * enqueues hist256 on the context stream and writes one row of 258 int64 to
 * device memory d_row: [0, 256) the job's weights, [256] its last min(8, n)
 * input bytes packed little-endian, [257] their count. The caller all-gathers
 * the rows (RCCL, same stream order) and passes them to huff_enc_pack_shards
 * (as hists / tails), which also takes this job's weights from hists[rank]. */
int huff_enc_hist_row(huff_enc* e, int64_t* d_row);
/* Total bits the tree assigns to this job (needs huff_enc_hist first). */
int huff_enc_bits(huff_enc* e, const huff_tree* t, uint64_t* total_bits);
/* pass 2: pack. The job's first symbol starts at global stream bit `bit_base`;
 * d_out[0] is the global byte bit_base/8. prev_tail (host, <= 8 bytes) are the
 * input bytes that immediately precede this job in the global stream (another
 * shard's tail) so the shared first byte is complete; NULL/0 when bit_base%8
 * == 0 or there is nothing before. Writes ceil((bit_base%8 + bits)/8) bytes,
 * the last one zero-padded. Also builds the restart index for decode. */
int huff_enc_pack(huff_enc* e, const huff_tree* t, uint64_t bit_base,
                  const uint8_t* prev_tail, size_t prev_tail_len,
                  uint8_t* d_out, size_t out_cap, uint64_t* total_bits);
/* Multi-shard pass 2 in one call: the job is shard `rank` of
 * `world` contiguous shards of one stream. hists = world x 256 per-shard
 * weights (the exchanged huff_enc_hist results), tails = world x 8 bytes where
 * shard q's last tail_lens[q] (<= 8) input bytes sit at tails[q*8 ...]. Builds
 * the tree of the summed weights (ByteWeights::from_bytes of the whole
 * stream), this shard's bit base (exclusive sum of the shards' bits) and
 * previous-tail bytes, and packs as huff_enc_pack. *tree_out receives the tree
 * (free with huff_tree_free). world = 1 is the single-GPU encode. On
 * HUFF_E_BUFFER_TOO_SMALL *bits_out still holds the bits needed. */
int huff_enc_pack_shards(huff_enc* e, const uint64_t* hists, uint32_t world, uint32_t rank,
                         const uint8_t* tails, const uint8_t* tail_lens,
                         uint8_t* d_out, size_t out_cap, huff_tree** tree_out,
                         uint64_t* bit_base_out, uint64_t* bits_out);
/* compress() on a resident buffer in one call (comp.rs:391-397 + the tree of
 * ByteWeights::from_bytes, weights.rs:265-279): pass 1, the host tree of
 * the job's weights, pass 2 at bit 0 — no caller code between the passes.
 * *tree_out receives the tree (free with huff_tree_free); on
 * HUFF_E_BUFFER_TOO_SMALL *bits_out still holds the bits needed. */
int huff_enc_compress(huff_enc* e, uint8_t* d_out, size_t out_cap, huff_tree** tree_out, uint64_t* bits_out);
/* Block-parallel decode of what huff_enc_pack wrote (same job, same tree),
 * using its restart index: d_comp is the pack's d_out, d_out gets n bytes. */
int huff_enc_decode(huff_enc* e, const huff_tree* t, const uint8_t* d_comp, uint8_t* d_out);

/* ------------------------------------------------------------------------ */
/* multi-GPU: sharded compress over an RCCL communicator  */
/* ------------------------------------------------------------------------ */
/* One process (or thread) per GPU, each with its own huff_ctx. The RCCL
 * communicator (xGMI) lives next to the context; rank 0 makes the id and the
 * caller hands its bytes to every rank over any channel it has. */
#define HUFF_COMM_ID_BYTES 128
typedef struct huff_comm huff_comm;
int huff_comm_unique_id(uint8_t id[HUFF_COMM_ID_BYTES]);
/* collective: every rank of `world` calls it with the same id; blocks until all joined */
int huff_comm_init(huff_ctx* ctx, const uint8_t id[HUFF_COMM_ID_BYTES], int world, int rank, huff_comm** out);
void huff_comm_free(huff_comm* c);
int huff_comm_world(const huff_comm* c, int* world, int* rank);
/* Collective sharded compress (replaces huff/src/comp.rs:161-172 + weights.rs:
 * 293-319, the per-part weights merged into ByteWeights of the whole input):
 * job `e` (a huff_enc of this rank's context) is shard `rank` of `world`
 * contiguous shards of one stream. Pass 1 on the shard, ONE ncclAllGather of a
 * 258 x int64 row per rank (weights + last <= 8 input bytes) on the context
 * stream, the tree of the summed weights on the host (identical on every
 * rank), this shard's bit base (sum of the previous shards' bits) and pass 2
 * at that base. Writes ceil((bit_base%8 + bits)/8) bytes at d_out; d_out[0]
 * is global stream byte bit_base/8. *owned_bytes_out = the prefix of d_out
 * this rank contributes to the concatenated stream (its partial last byte is
 * completed and owned by rank + 1; the last rank owns its zero-padded final
 * byte): the ranks' owned prefixes, concatenated in rank order, are
 * compress_with_tree over the whole stream (comp.rs:419-451). Decode the
 * shard with huff_enc_decode(e, *tree_out, d_out, ...). On
 * HUFF_E_BUFFER_TOO_SMALL *bits_out / *bit_base_out still hold the need. */
int huff_mgpu_compress(huff_comm* c, huff_enc* e, uint8_t* d_out, size_t out_cap, huff_tree** tree_out,
                       uint64_t* bit_base_out, uint64_t* bits_out, uint64_t* owned_bytes_out);
/* The exchange of the job's NEXT huff_mgpu_compress (pass 1, its row, the
 * all-gather, the rows' copy to the host) queued now, without waiting: the
 * next huff_mgpu_compress of this job only waits for the rows. Queued
 * between a job's pack and its decode, that wait and the host tree overlap
 * the decode (a streaming encoder's software pipeline; no reference
 * counterpart). Every rank must call it at the same point, as any
 * collective; one pending exchange per communicator (HUFF_E_STATE). */
int huff_mgpu_exchange_launch(huff_comm* c, huff_enc* e);
/* The host half of huff_mgpu_compress, for a caller that exchanges the rows
 * over its own channel: rows = world x 258 int64 in rank order, each what
 * huff_enc_hist_row wrote for that rank's shard (host memory, already
 * gathered); e is this rank's job after huff_enc_hist_row. Unpacks the rows
 * (weights, tail bytes; a tail count < 0 marks a rank that failed before the
 * exchange and makes every rank return HUFF_E_INVALID_ARG), builds the tree of
 * the summed weights, this shard's bit base and shared first byte, and packs
 * as huff_mgpu_compress does; same outputs. A rank whose pass 1 cannot run
 * still joins huff_mgpu_compress's collective with such a failed row, so no
 * rank is left blocked in it. */
int huff_mgpu_pack_rows(huff_enc* e, const int64_t* rows, int world, int rank, uint8_t* d_out, size_t out_cap,
                        huff_tree** tree_out, uint64_t* bit_base_out, uint64_t* bits_out,
                        uint64_t* owned_bytes_out);

/* decompress (comp.rs:487-519) of a device-resident stream that has no
 * restart index (e.g. written by the reference CPU path): comp_bytes bytes at
 * d_comp (any alignment; a stream not 16-B aligned is first copied to an
 * aligned buffer of the context), the last holding `padding` pad bits (the walk reads
 * 8 - padding bits of it; an incomplete final code is dropped). Self-
 * synchronising parallel decode; writes the letters to d_out and their count
 * to *n_out (set also on HUFF_E_BUFFER_TOO_SMALL; d_out NULL: count only). */
int huff_dev_decompress(huff_ctx* ctx, const huff_tree* t, const uint8_t* d_comp, size_t comp_bytes,
                        uint8_t padding, uint8_t* d_out, size_t out_cap, size_t* n_out);

/* Many small byte streams at once (device pointers, one
 * launch each, synchronous):
 *  huff_batch_hist:  d_hist[s][256] = the byte weights (ByteWeights::
 *                    from_bytes, weights.rs:265-279) of stream s =
 *                    d_in[d_offsets[s], d_offsets[s + 1]) (any length; an
 *                    offset pair with d_offsets[s + 1] < d_offsets[s] counts
 *                    as an empty stream).
 *  huff_batch_trees: HuffTree::from_weights of each d_hist[s] (tree_inner.rs:
 *                    281-320, with the reference's exact BinaryHeap tie order)
 *                    -> d_tree_bits + s * tree_stride: as_bin (tree_inner.rs:
 *                    632-663), MSB first, d_tree_nbits[s] bits; d_codes[s][l] =
 *                    code << 8 | len of letter l (0: no code); d_max_len[s];
 *                    d_status[s] = HUFF_OK, HUFF_E_EMPTY_WEIGHTS (all weights
 *                    zero: "provided empty weights"), HUFF_E_CODE_TOO_LONG (a
 *                    code longer than 56 bits: its d_codes entry is 0; the
 *                    tree bits are complete) or HUFF_E_INVALID_ARG (the
 *                    stream's weights sum to 2^54 or more, counting the byte-0
 *                    re-yield: no tree, 0 tree bits). tree_stride >=
 *                    HUFF_TREE_BITS_MAX_BYTES. */
#define HUFF_TREE_BITS_MAX_BYTES 322
int huff_batch_hist(huff_ctx* ctx, const uint8_t* d_in, const uint64_t* d_offsets, uint32_t nstreams,
                    uint64_t* d_hist);
int huff_batch_trees(huff_ctx* ctx, const uint64_t* d_hist, uint32_t nstreams, uint8_t* d_tree_bits,
                     size_t tree_stride, uint32_t* d_tree_nbits, uint64_t* d_codes, uint32_t* d_max_len,
                     uint32_t* d_status);

/* synthetic inputs generated on the device (not reference functions):
 * kind 0 = uniform bytes, 1 = Zipf(alpha) with cdf[256] (host), 2 = text.
 * Byte i of the stream depends only on (kind, seed, offset + i). */
int huff_dev_generate(huff_ctx* ctx, int kind, uint64_t seed, uint64_t offset, const uint64_t* cdf,
                      uint8_t* d_out, size_t n);

/* HBM calibration (measurement only, not a reference function): best-of-
 * `iters` GB/s (1e9) of a streaming 16-B nontemporal read of n bytes at d_src
 * and of a streaming copy d_src -> d_dst (2n bytes moved); both 16-B aligned.
 * bench.py's measured ceilings beside the 8 TB/s spec peak. */
int huff_dev_calibrate(huff_ctx* ctx, const uint8_t* d_src, uint8_t* d_dst, size_t n, int iters,
                       double* read_gbps, double* copy_gbps);

/* device memory helpers for callers without another allocator */
int huff_dev_alloc(huff_ctx* ctx, size_t bytes, void** d_ptr);
int huff_dev_free(huff_ctx* ctx, void* d_ptr);
int huff_memcpy_htod(huff_ctx* ctx, void* d_dst, const void* src, size_t bytes);
int huff_memcpy_dtoh(huff_ctx* ctx, void* dst, const void* d_src, size_t bytes);

/* ------------------------------------------------------------------------ */
/* huff CLI file path — huff/src/comp.rs:32-157                              */
/* ------------------------------------------------------------------------ */
/* read_compress_write: `.hff` = [pad byte][u32 BE tree len][tree][data].
 * block_size as the CLI's -b (default 2,000,000,000). Blocks after the first
 * are stitched exactly as the reference does (huff/src/comp.rs:196-201,
 * bug-compatible). */
int huff_file_compress(huff_ctx* ctx, const char* src_path, const char* dst_path, size_t block_size);
/* read_decompress_write (huff/src/comp.rs:79-157, :232-280) */
int huff_file_decompress(huff_ctx* ctx, const char* src_path, const char* dst_path, size_t block_size);
/* cli.rs:79-114 parse_block_size ("2G", "64Ki", ...): HUFF_E_INVALID_ARG on error */
int huff_parse_block_size(const char* s, size_t* out);

#ifdef __cplusplus
}
#endif
#endif /* HUFFGPU_H */
