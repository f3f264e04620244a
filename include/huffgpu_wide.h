/*
 * huffgpu_wide.h — C ABI for the reference's wider integer letters
 * (SURVEY.md §8f-3): HuffTree<L>, build_weights_map, compress_with_tree and
 * decompress for L in {u8,u16,u32,u64,u128, i8,i16,i32,i64,i128,usize,isize}
 * (letter.rs:41-60 integer_letter_impl, the HuffLetterAsBytes types).
 *
 * Conventions are those of huffgpu.h (int status, huff_last_error()). A
 * letter type is named by its width in bytes (1, 2, 4, 8, 16); letters cross
 * the ABI as arrays of that width in native (little-endian) integer layout, so
 * a Rust &[i32] is passed as (ptr, len) with width 4. Signed and unsigned
 * types of one width share the code: the reference converts letters with
 * to_be_bytes / from_be_bytes, which are bit copies.
 *
 * Ordering. HuffTree::from_weights (tree_inner.rs:281-320) depends on the
 * order its Weights iterate in. The reference's HashMap weights
 * (weights.rs:82-123) iterate in RandomState order, so huff_wtree_from_weights
 * takes the (letter, weight) pairs in the caller's iteration order and is
 * exact for it; huff_wweights_map returns ascending letter order.
 */
#ifndef HUFFGPU_WIDE_H
#define HUFFGPU_WIDE_H

#include "huffgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct huff_wtree huff_wtree;
typedef struct huff_wcompress_data huff_wcompress_data;
typedef struct huff_wenc huff_wenc;

/* ---------------- HuffTree<L> (host; tree_inner.rs) ---------------------- */
/* HuffTree::from_weights (tree_inner.rs:281-320) over n pairs in iteration
 * order; HUFF_E_EMPTY_WEIGHTS for n == 0 (the reference panics). */
int huff_wtree_from_weights(uint32_t width, const void* letters, const uint64_t* weights, size_t n,
                            huff_wtree** out);
int huff_wtree_clone(const huff_wtree* t, huff_wtree** out);
void huff_wtree_free(huff_wtree* t);
uint32_t huff_wtree_width(const huff_wtree* t);
size_t huff_wtree_num_leaves(const huff_wtree* t);
/* HuffTree::read_codes (tree_inner.rs:356-440): one entry per distinct
 * letter, ascending letter value; code right-aligned, len in bits. *count is
 * set to the number of entries even when cap is short (BUFFER_TOO_SMALL).
 * HUFF_E_CODE_TOO_LONG if a code exceeds 64 bits. */
int huff_wtree_read_codes(const huff_wtree* t, void* letters, uint64_t* code, uint8_t* len, size_t cap,
                          size_t* count);
/* HuffTree::as_bin (tree_inner.rs:632-668): W*8 bits per letter, packed
 * Msb0 into ceil(nbits/8) bytes (out may be NULL to query *nbits). */
int huff_wtree_as_bin(const huff_wtree* t, uint8_t* out, size_t cap, size_t* nbits);
/* HuffTree::<L>::try_from_bin (tree_inner.rs:522-604); FromBinError
 * messages "Provided BitVec is too small/big for an encoded HuffTree". */
int huff_wtree_try_from_bin(uint32_t width, const uint8_t* bits, size_t nbits, huff_wtree** out);
/* Walking the tree, as huffgpu.h's huff_tree_root / huff_branch_* for u8
 * (HuffTree::root tree_inner.rs:322-325, HuffBranch branch.rs:207-279,
 * HuffLeaf leaf.rs:61-73): node ids >= 0, -1 = None; the letter as W
 * little-endian bytes. */
int huff_wtree_root(const huff_wtree* t, int32_t* branch);
int huff_wbranch_children(const huff_wtree* t, int32_t branch, int32_t* left, int32_t* right);
int huff_wbranch_leaf(const huff_wtree* t, int32_t branch, int* has_letter, void* letter, uint64_t* weight);
int huff_wbranch_code(const huff_wtree* t, int32_t branch, uint8_t* bits, size_t cap, size_t* nbits,
                      int* has_code);

/* ---------------- weights (GPU) ------------------------------------------ */
/* build_weights_map (weights.rs:82-123) of n host letters: the distinct
 * letters (ascending) and their counts; *count as in read_codes. */
int huff_wweights_map(huff_ctx* ctx, uint32_t width, const void* letters, size_t n, void* letters_out,
                      uint64_t* weights_out, size_t cap, size_t* count);

/* ---------------- CompressData<L> (comp.rs:40-300) ----------------------- */
int huff_wcd_new(const uint8_t* comp, size_t len, uint8_t padding, const huff_wtree* t, huff_wcompress_data** out);
void huff_wcd_free(huff_wcompress_data* cd);
int huff_wcd_comp_bytes(const huff_wcompress_data* cd, const uint8_t** ptr, size_t* len);
uint8_t huff_wcd_padding(const huff_wcompress_data* cd);
const huff_wtree* huff_wcd_tree(const huff_wcompress_data* cd);
int huff_wcd_has_index(const huff_wcompress_data* cd);
/* CompressData::to_bytes (comp.rs:279-300) with the W*8-bit tree */
int huff_wcd_to_bytes(const huff_wcompress_data* cd, uint8_t* out, size_t cap, size_t* out_len);
/* CompressData::<L>::try_from_bytes (comp.rs:128-184) */
int huff_wcd_try_from_bytes(uint32_t width, const uint8_t* bytes, size_t n, huff_wcompress_data** out);

/* ---------------- compress / decompress (GPU, host buffers) -------------- */
/* compress_with_tree (comp.rs:419-451) of n letters of the tree's width;
 * HUFF_E_MISSING_LETTER for the first letter without a code (input order),
 * its value via huff_last_missing_wletter. The tree is borrowed. */
int huff_wcompress_with_tree(huff_ctx* ctx, const void* letters, size_t n, const huff_wtree* t,
                             huff_wcompress_data** out);
/* compress (comp.rs:353-359): build_weights_map order as huff_wweights_map */
int huff_wcompress(huff_ctx* ctx, uint32_t width, const void* letters, size_t n, huff_wcompress_data** out);
/* decompress (comp.rs:487-519) into cap letters; *n_out = letters decoded
 * (BUFFER_TOO_SMALL when cap is short). Without a restart index (data from
 * try_from_bytes / huff_wcd_new) the self-synchronising decoder runs. */
int huff_wdecompress(huff_ctx* ctx, const huff_wcompress_data* cd, void* out, size_t cap, size_t* n_out);
/* the letter of the last HUFF_E_MISSING_LETTER of a wide call (width bytes) */
int huff_last_missing_wletter(void* out16, uint32_t* width);

/* ---------------- device-resident job (bench / HBM-resident data) -------- */
/* d_in: n letters of `width` bytes in HBM, 16-byte aligned */
int huff_wenc_create(huff_ctx* ctx, uint32_t width, const void* d_in, size_t n, huff_wenc** out);
void huff_wenc_free(huff_wenc* e);
/* pass A: code lengths, restart index; *total_bits */
int huff_wenc_bits(huff_wenc* e, const huff_wtree* t, uint64_t* total_bits);
/* pass B into d_out (any alignment, out_cap >= ceil(bits / 8)) */
int huff_wenc_pack(huff_wenc* e, const huff_wtree* t, uint8_t* d_out, size_t out_cap, uint64_t* total_bits);
/* restart-index decode of this job's pack output into d_out (n * width bytes);
 * d_comp at any alignment (a stream not 16-B aligned is first copied to an
 * aligned buffer of the context) */
int huff_wenc_decode(huff_wenc* e, const huff_wtree* t, const uint8_t* d_comp, uint8_t* d_out);
/* self-synchronising decode of a device stream (no index), d_comp at any
 * alignment (as huff_wenc_decode): returns the count in *n_out; d_out NULL =
 * count only */
int huff_dev_wdecompress(huff_ctx* ctx, const huff_wtree* t, const uint8_t* d_comp, size_t comp_bytes,
                         uint8_t padding, void* d_out, size_t out_cap_letters, size_t* n_out);

#ifdef __cplusplus
}
#endif

#endif /* HUFFGPU_WIDE_H */
