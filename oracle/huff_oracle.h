/*
 * huff_oracle.h — CPU ORACLE for the huff-encoding hot path.
 *
 * TEST INFRASTRUCTURE ONLY. Nothing in the product (huff-encoding_amd/) links,
 * loads or calls this code. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / the timed CPU restatement.
 *
 * It is a plain-C restatement of the reference Rust crate k-xlsx/huff-encoding
 * (read-only at /root/reference). Every function cites the reference file:line
 * it follows. The reference is Rust and no Rust toolchain exists in this image,
 * so the reference cannot be built (oracle/_ref is therefore absent; see
 * DESIGN.md "Oracle"). The restatement is pinned by the reference's own doctest
 * and test known answers (tests/golden/reference_pinned.json).
 *
 * Bit vectors (bitvec::BitVec<Msb0,u8>) are modelled as arrays holding one bit
 * per byte (0/1), the most literal form of the reference's per-bit loops.
 */
#ifndef HUFF_ORACLE_H
#define HUFF_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (mirror include/huffgpu.h so tests can compare directly) */
enum {
    ORC_OK = 0,
    ORC_E_EMPTY_WEIGHTS = 2,     /* tree_inner.rs:283-285 panic "provided empty weights" */
    ORC_E_MISSING_LETTER = 3,    /* comp.rs:426-432 CompressError                       */
    ORC_E_FROM_BIN = 4,          /* tree_inner.rs:530-590 FromBinError                  */
    ORC_E_FROM_BYTES = 5,        /* comp.rs:128-184 CompressedDataFromBytesError        */
    ORC_E_BUFFER = 6,            /* caller buffer too small                             */
    ORC_E_EMPTY_COMP = 14,       /* comp.rs:56-58 panic "provided comp_bytes are empty" */
    ORC_E_PADDING = 15,          /* comp.rs:59-61 panic "padding bits ... larger than 7"*/
    ORC_E_TREE_LEN = 16,         /* comp.rs:153-155 panic "stored tree length ... 2"   */
    ORC_E_MISSING_HEADER = 11,   /* huff/src/comp.rs:95-100,123-128                    */
    ORC_E_INVALID_HEADER = 12,   /* huff/src/comp.rs:107-112,141-144                   */
};

/* ---------------- weights.rs: ByteWeights ---------------- */
typedef struct {
    uint64_t w[256];   /* weights.rs:176  weights: [usize; 256] */
    uint64_t len;      /* weights.rs:177  len: usize (distinct count) */
} orc_weights;

void   orc_weights_new(orc_weights* bw);
void   orc_weights_from_bytes(const uint8_t* bytes, size_t n, orc_weights* out);
size_t orc_weights_iter(const orc_weights* bw, uint8_t letter[257], uint64_t weight[257]);
void   orc_weights_add(orc_weights* self, const orc_weights* other);
void   orc_weights_threaded(const uint8_t* bytes, size_t n, size_t thread_num, orc_weights* out);

/* ---------------- tree/: HuffTree ---------------- */
typedef struct orc_tree orc_tree;

/* leaves pushed in the given order (letters are opaque ids) */
orc_tree* orc_tree_from_leaves(const uint64_t* letters, const uint64_t* weights, size_t n);
/* NULL when weights are empty (the reference panics) */
orc_tree* orc_tree_from_weights(const orc_weights* bw);
void      orc_tree_free(orc_tree* t);
size_t    orc_tree_num_leaves(const orc_tree* t);

/* read_codes for letters < nletters; code bits are one bit per byte, row stride
 * `stride`; code_len[l] = 0 when l has no code. Overwrite semantics of the
 * HashMap insert order are reproduced. Returns max code length. */
uint32_t orc_tree_codes(const orc_tree* t, uint32_t nletters, uint8_t* code_bits,
                        size_t stride, uint32_t* code_len);

/* as_bin: one bit per byte; returns the number of bits (bits may be NULL) */
size_t orc_tree_as_bin(const orc_tree* t, uint32_t letter_bits, uint8_t* bits);
/* try_from_bin: returns ORC_OK or ORC_E_FROM_BIN (msg set) */
int orc_tree_try_from_bin(const uint8_t* bits, size_t nbits, uint32_t letter_bits,
                          orc_tree** out, const char** msg);

/* ---------------- comp.rs ---------------- */
/* compress_with_tree; out must hold >= ceil(sum bits/8); returns ORC_OK,
 * ORC_E_MISSING_LETTER (missing set), ORC_E_EMPTY_COMP (n==0 -> empty bytes). */
int orc_compress_with_tree(const uint8_t* in, size_t n, const orc_tree* t,
                           uint8_t* out, size_t cap, size_t* out_len,
                           uint8_t* padding, uint8_t* missing);
/* total bits the tree's codes assign to `in` (helper for buffer sizing) */
uint64_t orc_compressed_bits(const uint8_t* in, size_t n, const orc_tree* t);
/* decompress; returns number of symbols (writes at most cap of them) */
size_t orc_decompress(const uint8_t* comp, size_t len, uint8_t padding,
                      const orc_tree* t, uint8_t* out, size_t cap);
/* CompressData::to_bytes; returns bytes needed (writes if cap suffices) */
size_t orc_to_bytes(const uint8_t* comp, size_t len, uint8_t padding,
                    const orc_tree* t, uint8_t* out, size_t cap);
/* CompressData::try_from_bytes; comp_off/comp_len index into bytes */
int orc_try_from_bytes(const uint8_t* bytes, size_t n, orc_tree** tree,
                       uint8_t* padding, size_t* comp_off, size_t* comp_len,
                       const char** msg);

/* ---------------- huff/src/comp.rs: the CLI file path (in memory) ---------------- */
int orc_cli_compress(const uint8_t* file, size_t n, size_t block_size,
                     uint8_t* out, size_t cap, size_t* out_len);
int orc_cli_decompress(const uint8_t* hff, size_t n, size_t block_size,
                       uint8_t* out, size_t cap, size_t* out_len);
/* compress_with_tree / decompress over u64 letters (the wider integer
 * HuffLetterAsBytes types, letter.rs:41-60; trees from orc_tree_from_leaves
 * or orc_tree_try_from_bin with letter_bits = 8 * width) */
int orc_wcompress_with_tree(const uint64_t* in, size_t n, const orc_tree* t,
                            uint8_t* out, size_t cap, size_t* out_len,
                            uint8_t* padding, size_t* missing_idx);
size_t orc_wdecompress(const uint8_t* comp, size_t len, uint8_t padding,
                       const orc_tree* t, uint64_t* out, size_t cap);
/* huff/src/utils.rs:2-25 */
size_t orc_offset_bytes(const uint8_t* bytes, size_t n, size_t shift, uint8_t* out);

/* ---------------- table-driven checker (large sizes) ----------------
 * Not a restatement: a fast, multithreaded encoder used to check the GPU at
 * full BASELINE sizes. Validated bit-exact against orc_compress_with_tree
 * by tests/test_oracle.py. code[] is right-aligned, len in bits (<= 64). */
int orc_fast_encode(const uint8_t* in, size_t n, const uint64_t code[256],
                    const uint8_t len[256], int threads, uint64_t bit_base,
                    uint8_t* out, size_t cap, uint64_t* total_bits);
/* as orc_fast_encode, also writing each job's absolute start bit (the job
 * split: threads clamped to n/4096+1, job i = [i*(n/T), (i+1)*(n/T)), the last
 * takes the remainder) into job_start[T] when non-NULL */
int orc_fast_encode_idx(const uint8_t* in, size_t n, const uint64_t code[256],
                        const uint8_t len[256], int threads, uint64_t bit_base,
                        uint8_t* out, size_t cap, uint64_t* total_bits, uint64_t* job_start);
/* table-driven multithreaded decode of n letters over that job split */
int orc_fast_decode(const uint8_t* comp, size_t comp_bytes, const orc_tree* t, size_t n,
                    int threads, const uint64_t* job_start, uint8_t* out);
void orc_fast_hist(const uint8_t* in, size_t n, int threads, uint64_t w[256]);

/* ---------------- synthetic inputs (not reference code) ---------------- */
uint64_t orc_splitmix64(uint64_t state_index, uint64_t seed);
void orc_gen_uniform(uint64_t seed, uint64_t offset, size_t n, uint8_t* out);
void orc_zipf_cdf(double alpha, uint64_t cdf[256]);
void orc_gen_zipf(uint64_t seed, uint64_t offset, size_t n, const uint64_t cdf[256], uint8_t* out);
void orc_gen_text(uint64_t seed, uint64_t offset, size_t n, uint8_t* out);

/* ---------------- timing helper for bench.py cpu_baseline ---------------- */
double orc_now(void);

#ifdef __cplusplus
}
#endif
#endif
