/*
 * huff_oracle.c — CPU ORACLE (test infrastructure only; see huff_oracle.h).
 *
 * Plain-C restatement of k-xlsx/huff-encoding. Citations are relative to
 * /root/reference. Where the reference depends on Rust std / bitvec 0.20.1
 * semantics (BinaryHeap sift order, Msb0 bit order), the restated algorithm
 * is written out and cited to the call site that depends on it.
 */
#include "huff_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ======================================================================== */
/* weights.rs — ByteWeights                                                  */
/* ======================================================================== */

/* weights.rs:245-250 ByteWeights::new */
void orc_weights_new(orc_weights* bw) { memset(bw, 0, sizeof(*bw)); }

/* weights.rs:265-279 ByteWeights::from_bytes: one increment per byte,
 * len counts bins that went 0 -> 1. */
void orc_weights_from_bytes(const uint8_t* bytes, size_t n, orc_weights* out)
{
    orc_weights_new(out);
    for (size_t i = 0; i < n; ++i) {
        if (out->w[bytes[i]] == 0) out->len += 1;
        out->w[bytes[i]] += 1;
    }
}

/* weights.rs:323-329 ByteWeights::get: None for a zero weight */
static int bw_get(const orc_weights* bw, size_t idx_u8) { return bw->w[idx_u8 & 0xFF] != 0; }

/* weights.rs:423-441 Iter::next (identical to IntoIter::next, :396-415).
 * Walks current_index 0..256; the `as u8` cast in get() makes index 256 read
 * byte 0, so when byte 0 is present and byte 255 absent the iterator yields
 * (0, w[0]) a second time at the end. Returns the count. */
size_t orc_weights_iter(const orc_weights* bw, uint8_t letter[257], uint64_t weight[257])
{
    size_t cur = 0, count = 0;
    for (;;) {
        /* if self.current_index == 256 { return None } */
        if (cur == 256) break;
        /* while self.weights.get(&(cur as u8)).is_none() { if cur == 256 {None}; cur += 1 } */
        int stop = 0;
        while (!bw_get(bw, cur)) {
            if (cur == 256) { stop = 1; break; }
            cur += 1;
        }
        if (stop) break;
        letter[count] = (uint8_t)(cur & 0xFF);
        weight[count] = bw->w[cur & 0xFF];
        count += 1;
        /* if self.current_index != 256 { self.current_index += 1; } */
        if (cur != 256) cur += 1;
    }
    return count;
}

/* weights.rs:374-387 add_byte_weights: iterate `other` with Iter (so the
 * wrap duplicate of byte 0 is added twice). */
void orc_weights_add(orc_weights* self, const orc_weights* other)
{
    uint8_t l[257];
    uint64_t f[257];
    size_t cnt = orc_weights_iter(other, l, f);
    for (size_t i = 0; i < cnt; ++i) {
        if (self->w[l[i]] != 0) {
            self->w[l[i]] += f[i];
        } else {
            self->w[l[i]] = f[i];
            self->len += 1;
        }
    }
}

/* utils.rs:6-28 ration_vec: T rations of n/T elements, the last takes the
 * remainder; when n/T == 0 a single ration with everything. Each ration is
 * copied (`.to_vec()`, utils.rs:12,20,23) — the copy is reproduced. */
typedef struct { uint8_t* data; size_t n; orc_weights res; } ration_job;

static void* ration_worker(void* p)
{
    ration_job* j = (ration_job*)p;
    orc_weights_from_bytes(j->data, j->n, &j->res); /* weights.rs:300-302 */
    return NULL;
}

/* weights.rs:293-319 threaded_from_bytes: spawn one thread per ration, join
 * in order, then `weights = vec.pop(); for other in vec { weights += other }`
 * i.e. the LAST ration's weights absorb rations 0..T-2 in order. */
void orc_weights_threaded(const uint8_t* bytes, size_t n, size_t thread_num, orc_weights* out)
{
    size_t per = thread_num ? n / thread_num : 0;
    size_t nr = (per == 0) ? 1 : thread_num;
    ration_job* jobs = (ration_job*)calloc(nr, sizeof(ration_job));
    pthread_t* th = (pthread_t*)calloc(nr, sizeof(pthread_t));
    size_t cur = 0;
    for (size_t i = 0; i < nr; ++i) {
        size_t len = (per == 0) ? n : ((i == nr - 1) ? n - cur : per);
        jobs[i].data = (uint8_t*)malloc(len ? len : 1);
        if (len) memcpy(jobs[i].data, bytes + cur, len);
        jobs[i].n = len;
        cur += len;
    }
    for (size_t i = 0; i < nr; ++i) pthread_create(&th[i], NULL, ration_worker, &jobs[i]);
    for (size_t i = 0; i < nr; ++i) pthread_join(th[i], NULL);
    *out = jobs[nr - 1].res;
    for (size_t i = 0; i + 1 < nr; ++i) orc_weights_add(out, &jobs[i].res);
    for (size_t i = 0; i < nr; ++i) free(jobs[i].data);
    free(jobs);
    free(th);
}

/* ======================================================================== */
/* tree/ — HuffTree                                                          */
/* ======================================================================== */

typedef struct {
    int leaf;           /* letter.is_some() */
    uint64_t letter;
    uint64_t weight;
    int32_t left, right; /* child node indices, -1 for none */
} orc_node;

struct orc_tree {
    orc_node* nodes;
    size_t nnodes, cap;
    int32_t root;
};

static int32_t tree_new_node(orc_tree* t, int leaf, uint64_t letter, uint64_t w, int32_t l, int32_t r)
{
    if (t->nnodes == t->cap) {
        t->cap = t->cap ? t->cap * 2 : 64;
        t->nodes = (orc_node*)realloc(t->nodes, t->cap * sizeof(orc_node));
    }
    orc_node* nd = &t->nodes[t->nnodes];
    nd->leaf = leaf; nd->letter = letter; nd->weight = w; nd->left = l; nd->right = r;
    return (int32_t)t->nnodes++;
}

void orc_tree_free(orc_tree* t)
{
    if (!t) return;
    free(t->nodes);
    free(t);
}

/* Rust std BinaryHeap<HuffBranchHeapItem> as used by branch_heap.rs:18-58.
 * HuffBranchHeapItem's Ord is reversed on weight only (branch_heap.rs:67-71,
 * leaf.rs:31-35), so "a <= b" (as the heap evaluates it) means a.w >= b.w.
 * The std algorithms (push -> sift_up; pop -> swap last into root, then
 * sift_down_to_bottom + sift_up) are written out below: tie order decides the
 * tree shape, hence the output bits. */
typedef struct { int32_t node; uint64_t w; } heap_item;

static int heap_le(heap_item a, heap_item b) { return a.w >= b.w; }

static size_t heap_sift_up(heap_item* d, size_t start, size_t pos)
{
    heap_item elem = d[pos];
    while (pos > start) {
        size_t parent = (pos - 1) / 2;
        if (heap_le(elem, d[parent])) break;  /* elem <= parent -> stop (ties stop) */
        d[pos] = d[parent];
        pos = parent;
    }
    d[pos] = elem;
    return pos;
}

static void heap_sift_down_to_bottom(heap_item* d, size_t end, size_t pos)
{
    size_t start = pos;
    heap_item elem = d[pos];
    size_t child = 2 * pos + 1;
    size_t lim = end >= 2 ? end - 2 : 0;   /* end.saturating_sub(2) */
    while (child <= lim && end >= 2) {
        if (heap_le(d[child], d[child + 1])) child += 1;  /* pick right on ties */
        d[pos] = d[child];
        pos = child;
        child = 2 * pos + 1;
    }
    if (end >= 1 && child == end - 1) {
        d[pos] = d[child];
        pos = child;
    }
    d[pos] = elem;
    heap_sift_up(d, start, pos);
}

static void heap_push(heap_item* d, size_t* len, heap_item x)
{
    d[*len] = x;
    *len += 1;
    heap_sift_up(d, 0, *len - 1);
}

static heap_item heap_pop(heap_item* d, size_t* len)
{
    *len -= 1;
    heap_item item = d[*len];
    if (*len > 0) {
        heap_item t = d[0];
        d[0] = item;
        item = t;
        heap_sift_down_to_bottom(d, *len, 0);
    }
    return item;
}

/* tree_inner.rs:281-320 HuffTree::from_weights with branch_heap.rs:52-58
 * build (leaves pushed in iterator order). */
orc_tree* orc_tree_from_leaves(const uint64_t* letters, const uint64_t* weights, size_t n)
{
    if (n == 0) return NULL; /* tree_inner.rs:283-285 panic("provided empty weights") */
    orc_tree* t = (orc_tree*)calloc(1, sizeof(orc_tree));
    heap_item* heap = (heap_item*)malloc(sizeof(heap_item) * (n + 1));
    size_t hl = 0;
    for (size_t i = 0; i < n; ++i) {
        heap_item it;
        it.node = tree_new_node(t, 1, letters[i], weights[i], -1, -1);
        it.w = weights[i];
        heap_push(heap, &hl, it);
    }
    while (hl > 1) {                                  /* tree_inner.rs:289 */
        heap_item mn = heap_pop(heap, &hl);           /* :291 min -> left  */
        heap_item nx = heap_pop(heap, &hl);           /* :292 next -> right */
        heap_item j;
        j.w = mn.w + nx.w;                            /* :298 */
        j.node = tree_new_node(t, 0, 0, j.w, mn.node, nx.node);
        heap_push(heap, &hl, j);                      /* :302 */
    }
    t->root = heap_pop(heap, &hl).node;               /* :306 */
    free(heap);
    return t;
}

orc_tree* orc_tree_from_weights(const orc_weights* bw)
{
    if (bw->len == 0) return NULL;                    /* is_empty() -> panic */
    uint8_t l[257];
    uint64_t w[257];
    uint64_t ll[257];
    size_t cnt = orc_weights_iter(bw, l, w);          /* into_iter order, §C.1 */
    for (size_t i = 0; i < cnt; ++i) ll[i] = l[i];
    return orc_tree_from_leaves(ll, w, cnt);
}

size_t orc_tree_num_leaves(const orc_tree* t)
{
    size_t c = 0;
    for (size_t i = 0; i < t->nnodes; ++i) c += t->nodes[i].leaf;
    return c;
}

/* tree_inner.rs:388-419 read_codes_with_hasher: codes of each leaf are its
 * path (left 0, right 1; tree_inner.rs:422-440); leaves are inserted in
 * left-to-right DFS order so a later leaf with the same letter overwrites an
 * earlier one. A root leaf gets code "0" (tree_inner.rs:313-315,416). */
typedef struct {
    uint32_t nletters;
    uint8_t* bits;
    size_t stride;
    uint32_t* len;
    uint8_t path[512];
    uint32_t maxlen;
} codes_ctx;

static void codes_rec(const orc_tree* t, int32_t nd, uint32_t depth, codes_ctx* c)
{
    const orc_node* n = &t->nodes[nd];
    if (n->leaf) {
        if (n->letter < c->nletters) {
            memcpy(c->bits + (size_t)n->letter * c->stride, c->path, depth);
            c->len[n->letter] = depth;
        }
        if (depth > c->maxlen) c->maxlen = depth;
        return;
    }
    c->path[depth] = 0;
    codes_rec(t, n->left, depth + 1, c);
    c->path[depth] = 1;
    codes_rec(t, n->right, depth + 1, c);
}

uint32_t orc_tree_codes(const orc_tree* t, uint32_t nletters, uint8_t* code_bits,
                        size_t stride, uint32_t* code_len)
{
    codes_ctx c;
    memset(&c, 0, sizeof(c));
    c.nletters = nletters; c.bits = code_bits; c.stride = stride; c.len = code_len;
    for (uint32_t i = 0; i < nletters; ++i) code_len[i] = 0;
    const orc_node* r = &t->nodes[t->root];
    if (r->leaf) {
        if (r->letter < nletters) {
            code_bits[(size_t)r->letter * stride] = 0;
            code_len[r->letter] = 1;
        }
        return 1;
    }
    codes_rec(t, t->root, 0, &c);
    return c.maxlen;
}

/* tree_inner.rs:632-668 as_bin: preorder, joint -> 1, leaf -> 0 + letter
 * big-endian (letter_bits bits, MSB first). */
static size_t as_bin_rec(const orc_tree* t, int32_t nd, uint32_t lb, uint8_t* bits, size_t pos)
{
    const orc_node* n = &t->nodes[nd];
    if (!n->leaf) {
        if (bits) bits[pos] = 1;
        pos += 1;
        pos = as_bin_rec(t, n->left, lb, bits, pos);
        return as_bin_rec(t, n->right, lb, bits, pos);
    }
    if (bits) bits[pos] = 0;
    pos += 1;
    for (uint32_t b = 0; b < lb; ++b) {
        uint32_t shift = lb - 1 - b;
        if (bits) bits[pos] = (shift < 64) ? (uint8_t)((n->letter >> shift) & 1) : 0;
        pos += 1;
    }
    return pos;
}

size_t orc_tree_as_bin(const orc_tree* t, uint32_t letter_bits, uint8_t* bits)
{
    return as_bin_rec(t, t->root, letter_bits, bits, 0);
}

/* tree_inner.rs:522-604 try_from_bin (recursive read_branches_from_bits). */
static const char* MSG_SMALL = "Provided BitVec is too small for an encoded HuffTree";
static const char* MSG_BIG = "Provided BitVec is too big for an encoded HuffTree";

static int from_bin_rec(orc_tree* t, const uint8_t* bits, size_t nbits, size_t* pos,
                        uint32_t lb, int32_t* out, const char** msg)
{
    if (*pos >= nbits) { *msg = MSG_SMALL; return ORC_E_FROM_BIN; }   /* :530-535 */
    uint8_t b = bits[(*pos)++];
    if (b) {                                                              /* joint */
        int32_t l, r;
        int e = from_bin_rec(t, bits, nbits, pos, lb, &l, msg);
        if (e) return e;
        e = from_bin_rec(t, bits, nbits, pos, lb, &r, msg);
        if (e) return e;
        *out = tree_new_node(t, 0, 0, 0, l, r);
        return ORC_OK;
    }
    if (nbits - *pos < lb) { *msg = MSG_SMALL; return ORC_E_FROM_BIN; }  /* :554-559 */
    uint64_t letter = 0;
    for (uint32_t i = 0; i < lb; ++i) {
        letter = (lb - i - 1 < 64) ? (letter << 1) | bits[*pos + i] : letter;
    }
    *pos += lb;
    *out = tree_new_node(t, 1, letter, 0, -1, -1);
    return ORC_OK;
}

int orc_tree_try_from_bin(const uint8_t* bits, size_t nbits, uint32_t letter_bits,
                          orc_tree** out, const char** msg)
{
    orc_tree* t = (orc_tree*)calloc(1, sizeof(orc_tree));
    size_t pos = 0;
    int32_t root;
    const char* m = NULL;
    int e = from_bin_rec(t, bits, nbits, &pos, letter_bits, &root, &m);
    if (!e && pos != nbits) { m = MSG_BIG; e = ORC_E_FROM_BIN; }        /* :586-590 */
    if (e) {
        orc_tree_free(t);
        if (msg) *msg = m;
        *out = NULL;
        return e;
    }
    t->root = root;
    *out = t;
    return ORC_OK;
}

/* ======================================================================== */
/* comp.rs                                                                   */
/* ======================================================================== */

/* utils.rs:37-40 calc_padding_bits */
static uint8_t calc_padding_bits(uint64_t bit_count)
{
    uint8_t n = (uint8_t)(8 - bit_count % 8);
    return n == 8 ? 0 : n;
}

#define CODE_STRIDE 512

/* comp.rs:419-451 compress_with_tree: per letter code lookup, per bit
 * `comp_byte |= bit << bit_ptr` from bit 7 down, flush at 0; padding =
 * bit_ptr==7 ? 0 : bit_ptr+1 and the partial byte is pushed if padding != 0. */
int orc_compress_with_tree(const uint8_t* in, size_t n, const orc_tree* t,
                           uint8_t* out, size_t cap, size_t* out_len,
                           uint8_t* padding, uint8_t* missing)
{
    uint8_t* codes = (uint8_t*)calloc(256, CODE_STRIDE);
    uint32_t lens[256];
    orc_tree_codes(t, 256, codes, CODE_STRIDE, lens);             /* :421 read_codes */
    size_t o = 0;
    uint8_t comp_byte = 0;
    int bit_ptr = 7;
    for (size_t i = 0; i < n; ++i) {
        uint8_t letter = in[i];
        if (lens[letter] == 0) {                                   /* :426-432 */
            if (missing) *missing = letter;
            free(codes);
            return ORC_E_MISSING_LETTER;
        }
        const uint8_t* code = codes + (size_t)letter * CODE_STRIDE;
        for (uint32_t b = 0; b < lens[letter]; ++b) {               /* :433-443 */
            comp_byte |= (uint8_t)(code[b] << bit_ptr);
            if (bit_ptr == 0) {
                if (o < cap) out[o] = comp_byte;
                o++;
                comp_byte = 0;
                bit_ptr = 7;
            } else {
                bit_ptr -= 1;
            }
        }
    }
    uint8_t pad = (bit_ptr == 7) ? 0 : (uint8_t)(bit_ptr + 1);    /* :446 */
    if (pad != 0) {                                                /* :447 */
        if (o < cap) out[o] = comp_byte;
        o++;
    }
    free(codes);
    *out_len = o;
    if (padding) *padding = pad;
    if (o == 0) return ORC_E_EMPTY_COMP;  /* CompressData::new panic, comp.rs:56-58 */
    return o > cap ? ORC_E_BUFFER : ORC_OK;
}

uint64_t orc_compressed_bits(const uint8_t* in, size_t n, const orc_tree* t)
{
    uint8_t* codes = (uint8_t*)calloc(256, CODE_STRIDE);
    uint32_t lens[256];
    orc_tree_codes(t, 256, codes, CODE_STRIDE, lens);
    uint64_t bits = 0;
    for (size_t i = 0; i < n; ++i) bits += lens[in[i]];
    free(codes);
    return bits;
}

/* comp.rs:487-519 decompress: bit-serial walk; a joint branch steps right on
 * 1 / left on 0; reaching a leaf emits and resets to the root. All bytes but
 * the last contribute 8 bits; the last contributes 8 - padding bits. */
typedef struct {
    const orc_tree* t;
    int32_t cur;
    uint8_t* out;
    size_t cap, count;
} walk_state;

static void walk_bits(walk_state* s, uint8_t byte, int nbits)
{
    const orc_node* nodes = s->t->nodes;
    for (int bit_ptr = 0; bit_ptr < nbits; ++bit_ptr) {
        if (!nodes[s->cur].leaf) {
            int bit = (byte >> (7 - bit_ptr)) & 1;
            s->cur = bit ? nodes[s->cur].right : nodes[s->cur].left;
        }
        if (nodes[s->cur].leaf) {
            if (s->count < s->cap) s->out[s->count] = (uint8_t)nodes[s->cur].letter;
            s->count++;
            s->cur = s->t->root;
        }
    }
}

size_t orc_decompress(const uint8_t* comp, size_t len, uint8_t padding,
                      const orc_tree* t, uint8_t* out, size_t cap)
{
    if (len == 0) return 0;
    walk_state s = {t, t->root, out, cap, 0};
    for (size_t i = 0; i + 1 < len; ++i) walk_bits(&s, comp[i], 8);
    walk_bits(&s, comp[len - 1], 8 - padding);
    return s.count;
}

/* ---- the same two functions for letters wider than a byte (u64 values;
 * letter.rs:41-60 integer types up to 64 bits) ---- */
typedef struct { uint64_t letter; uint32_t len; size_t order; uint8_t* bits; } wcode;

typedef struct { wcode* v; size_t n, cap; uint8_t* path; size_t path_cap; } wcodes_ctx;

static void wcodes_rec(const orc_tree* t, int32_t nd, uint32_t depth, wcodes_ctx* c)
{
    const orc_node* n = &t->nodes[nd];
    if (depth + 1 > c->path_cap) {
        c->path_cap = 2 * (depth + 1);
        c->path = (uint8_t*)realloc(c->path, c->path_cap);
    }
    if (n->leaf) {
        if (c->n == c->cap) {
            c->cap = c->cap ? 2 * c->cap : 64;
            c->v = (wcode*)realloc(c->v, c->cap * sizeof(wcode));
        }
        wcode* w = &c->v[c->n];
        w->letter = n->letter;
        w->len = depth;
        w->order = c->n;
        w->bits = (uint8_t*)malloc(depth ? depth : 1);
        memcpy(w->bits, c->path, depth);
        c->n++;
        return;
    }
    c->path[depth] = 0;
    wcodes_rec(t, n->left, depth + 1, c);
    c->path[depth] = 1;
    wcodes_rec(t, n->right, depth + 1, c);
}

static int wcode_cmp(const void* a, const void* b)
{
    const wcode* x = (const wcode*)a;
    const wcode* y = (const wcode*)b;
    if (x->letter != y->letter) return x->letter < y->letter ? -1 : 1;
    return x->order < y->order ? -1 : (x->order > y->order);
}

/* read_codes (tree_inner.rs:356-419): preorder inserts into a map, a later
 * leaf of the same letter overwriting; here: sorted by (letter, order) and the
 * last of each letter kept */
static size_t wcodes(const orc_tree* t, wcode** out)
{
    wcodes_ctx c;
    memset(&c, 0, sizeof(c));
    const orc_node* r = &t->nodes[t->root];
    if (r->leaf) {  /* tree_inner.rs:313-315: the root leaf's code is "0" */
        c.v = (wcode*)malloc(sizeof(wcode));
        c.v[0].letter = r->letter; c.v[0].len = 1; c.v[0].order = 0;
        c.v[0].bits = (uint8_t*)calloc(1, 1);
        *out = c.v;
        return 1;
    }
    wcodes_rec(t, t->root, 0, &c);
    free(c.path);
    qsort(c.v, c.n, sizeof(wcode), wcode_cmp);
    size_t k = 0;
    for (size_t i = 0; i < c.n; ++i) {
        if (i + 1 < c.n && c.v[i + 1].letter == c.v[i].letter) { free(c.v[i].bits); continue; }
        c.v[k++] = c.v[i];
    }
    *out = c.v;
    return k;
}

static const wcode* wfind(const wcode* v, size_t n, uint64_t letter)
{
    size_t lo = 0, hi = n;
    while (lo < hi) {
        size_t mid = (lo + hi) / 2;
        if (v[mid].letter < letter) lo = mid + 1; else hi = mid;
    }
    return (lo < n && v[lo].letter == letter) ? &v[lo] : NULL;
}

/* comp.rs:419-451 over u64 letters; ORC_E_MISSING_LETTER with the index of
 * the first letter (input order) that has no code */
int orc_wcompress_with_tree(const uint64_t* in, size_t n, const orc_tree* t,
                            uint8_t* out, size_t cap, size_t* out_len,
                            uint8_t* padding, size_t* missing_idx)
{
    wcode* v;
    size_t nv = wcodes(t, &v);
    size_t o = 0;
    uint8_t comp_byte = 0;
    int bit_ptr = 7, rc = ORC_OK;
    for (size_t i = 0; i < n; ++i) {
        const wcode* c = wfind(v, nv, in[i]);
        if (!c) {                                                  /* :426-432 */
            if (missing_idx) *missing_idx = i;
            rc = ORC_E_MISSING_LETTER;
            goto done;
        }
        for (uint32_t b = 0; b < c->len; ++b) {
            comp_byte |= (uint8_t)(c->bits[b] << bit_ptr);
            if (bit_ptr == 0) {
                if (o < cap) out[o] = comp_byte;
                o++;
                comp_byte = 0;
                bit_ptr = 7;
            } else {
                bit_ptr -= 1;
            }
        }
    }
    {
        uint8_t pad = (bit_ptr == 7) ? 0 : (uint8_t)(bit_ptr + 1);
        if (pad != 0) {
            if (o < cap) out[o] = comp_byte;
            o++;
        }
        *out_len = o;
        if (padding) *padding = pad;
        if (o == 0) rc = ORC_E_EMPTY_COMP;
        else if (o > cap) rc = ORC_E_BUFFER;
    }
done:
    for (size_t i = 0; i < nv; ++i) free(v[i].bits);
    free(v);
    return rc;
}

/* comp.rs:487-519 over u64 letters */
size_t orc_wdecompress(const uint8_t* comp, size_t len, uint8_t padding,
                       const orc_tree* t, uint64_t* out, size_t cap)
{
    if (len == 0) return 0;
    const orc_node* nodes = t->nodes;
    int32_t cur = t->root;
    size_t count = 0;
    for (size_t i = 0; i < len; ++i) {
        int nbits = (i + 1 < len) ? 8 : 8 - padding;
        for (int bp = 0; bp < nbits; ++bp) {
            if (!nodes[cur].leaf) cur = ((comp[i] >> (7 - bp)) & 1) ? nodes[cur].right : nodes[cur].left;
            if (nodes[cur].leaf) {
                if (count < cap) out[count] = nodes[cur].letter;
                count++;
                cur = t->root;
            }
        }
    }
    return count;
}

/* bitvec into_vec (Msb0): bit i -> byte i/8, mask 0x80 >> (i%8), zero tail */
static void pack_bits(const uint8_t* bits, size_t nbits, uint8_t* out)
{
    size_t nbytes = (nbits + 7) / 8;
    memset(out, 0, nbytes);
    for (size_t i = 0; i < nbits; ++i)
        if (bits[i]) out[i / 8] |= (uint8_t)(0x80 >> (i % 8));
}

/* comp.rs:279-300 to_bytes: [(tree_pad<<4)+data_pad][u32 BE tree_len][tree][comp] */
size_t orc_to_bytes(const uint8_t* comp, size_t len, uint8_t padding,
                    const orc_tree* t, uint8_t* out, size_t cap)
{
    size_t nb = orc_tree_as_bin(t, 8, NULL);
    uint8_t* bits = (uint8_t*)malloc(nb + 1);
    orc_tree_as_bin(t, 8, bits);
    uint8_t tpad = calc_padding_bits(nb);
    uint32_t tlen = (uint32_t)((nb + tpad) / 8);
    size_t need = 5 + (size_t)tlen + len;
    if (out && cap >= need) {
        out[0] = (uint8_t)((tpad << 4) + padding);
        out[1] = (uint8_t)(tlen >> 24); out[2] = (uint8_t)(tlen >> 16);
        out[3] = (uint8_t)(tlen >> 8);  out[4] = (uint8_t)tlen;
        pack_bits(bits, nb, out + 5);
        memcpy(out + 5 + tlen, comp, len);
    }
    free(bits);
    return need;
}

static const char* MSG_EMPTY = "slice is empty";
static const char* MSG_TLEN = "slice too short to read tree length";
static const char* MSG_TREE = "slice too short to read tree";
static const char* MSG_INVALID = "invalid tree in slice";

/* comp.rs:128-184 try_from_bytes */
int orc_try_from_bytes(const uint8_t* bytes, size_t n, orc_tree** tree,
                       uint8_t* padding, size_t* comp_off, size_t* comp_len,
                       const char** msg)
{
    *tree = NULL;
    if (n < 1) { *msg = MSG_EMPTY; return ORC_E_FROM_BYTES; }             /* :143 */
    uint8_t tpad = bytes[0] >> 4, dpad = bytes[0] & 0x0F;                  /* :144-145 */
    if (n < 5) { *msg = MSG_TLEN; return ORC_E_FROM_BYTES; }              /* :148-152 */
    size_t tlen = ((size_t)bytes[1] << 24) | ((size_t)bytes[2] << 16) |
                  ((size_t)bytes[3] << 8) | bytes[4];
    if (tlen < 2) { *msg = "stored tree length must be at least 2"; return ORC_E_TREE_LEN; }
    if (n < 5 + tlen) { *msg = MSG_TREE; return ORC_E_FROM_BYTES; }       /* :161 */
    size_t nbits = tlen * 8;
    uint8_t* bits = (uint8_t*)malloc(nbits);
    for (size_t i = 0; i < nbits; ++i) bits[i] = (bytes[5 + i / 8] >> (7 - i % 8)) & 1;
    nbits = tpad > nbits ? 0 : nbits - tpad;                               /* :164 pop */
    orc_tree* t = NULL;
    const char* m2;
    int e = orc_tree_try_from_bin(bits, nbits, 8, &t, &m2);
    free(bits);
    if (e) { *msg = MSG_INVALID; return ORC_E_FROM_BYTES; }               /* :167-177 */
    /* bytes.get(5+tree_len..) is Some(empty) at the end -> new() panics */
    if (n - (5 + tlen) == 0) {
        orc_tree_free(t);
        *msg = "provided comp_bytes are empty";
        return ORC_E_EMPTY_COMP;
    }
    if (dpad > 7) {                                                        /* comp.rs:59-61 */
        orc_tree_free(t);
        *msg = "padding bits cannot be larger than 7";
        return ORC_E_PADDING;
    }
    *tree = t;
    *padding = dpad;
    *comp_off = 5 + tlen;
    *comp_len = n - (5 + tlen);
    return ORC_OK;
}

/* ======================================================================== */
/* huff/src/comp.rs — the CLI file path, restated over in-memory files        */
/* ======================================================================== */

/* huff/src/utils.rs:2-25 offset_bytes: re-emit every bit of `bytes` starting
 * at bit_ptr = (7 - n) % 8 of the first output byte (after n/8 zero bytes). */
size_t orc_offset_bytes(const uint8_t* bytes, size_t n, size_t shift, uint8_t* out)
{
    size_t o = 0;
    for (size_t i = 0; i < shift / 8; ++i) out[o++] = 0;
    uint8_t comp_byte = 0;
    int bit_ptr = (int)((7 - shift) % 8);
    for (size_t i = 0; i < n; ++i) {
        for (int k = 0; k < 8; ++k) {
            comp_byte |= (uint8_t)(((bytes[i] >> (7 - k)) & 1) << bit_ptr);
            if (bit_ptr == 0) {
                out[o++] = comp_byte;
                comp_byte = 0;
                bit_ptr = 7;
            } else {
                bit_ptr -= 1;
            }
        }
    }
    int pad = bit_ptr == 7 ? 0 : bit_ptr + 1;
    if (pad != 0) out[o++] = comp_byte;
    return o;
}

typedef struct { uint8_t* d; size_t len, cap, pos; } membuf;

static void mb_write(membuf* m, const uint8_t* src, size_t n)
{
    if (m->pos + n > m->cap) {
        size_t nc = m->cap ? m->cap : 64;
        while (nc < m->pos + n) nc *= 2;
        m->d = (uint8_t*)realloc(m->d, nc);
        m->cap = nc;
    }
    memcpy(m->d + m->pos, src, n);
    m->pos += n;
    if (m->pos > m->len) m->len = m->pos;
}

/* huff/src/comp.rs:32-74 read_compress_write + :161-172 huff_tree_from_reader
 * + :177-227 compress_to_writer (multi-block stitching bug included, §C.3). */
int orc_cli_compress(const uint8_t* file, size_t n, size_t block_size,
                     uint8_t* out, size_t cap, size_t* out_len)
{
    /* pass 1: weights (huff_tree_from_reader) */
    orc_weights bw, part;
    orc_weights_new(&bw);
    size_t left = n, off = 0;
    while (left >= block_size) {                        /* read_exact(buf).is_ok() */
        orc_weights_threaded(file + off, block_size, 12, &part);   /* :164 */
        orc_weights_add(&bw, &part);
        off += block_size;
        left -= block_size;
    }
    if (left > 0) {                                     /* :167-169 */
        orc_weights_threaded(file + off, left, 12, &part);
        orc_weights_add(&bw, &part);
    }
    orc_tree* t = orc_tree_from_weights(&bw);           /* :171 */
    if (!t) return ORC_E_EMPTY_WEIGHTS;

    /* header (:47-59) */
    size_t nb = orc_tree_as_bin(t, 8, NULL);
    uint8_t* bits = (uint8_t*)malloc(nb + 1);
    orc_tree_as_bin(t, 8, bits);
    uint8_t tpad = calc_padding_bits(nb);
    size_t tbytes = (nb + 7) / 8;
    uint8_t* tb = (uint8_t*)malloc(tbytes + 1);
    pack_bits(bits, nb, tb);
    free(bits);

    membuf m = {0};
    uint8_t zero = 0;
    mb_write(&m, &zero, 1);
    uint8_t lb[4] = {(uint8_t)(tbytes >> 24), (uint8_t)(tbytes >> 16), (uint8_t)(tbytes >> 8), (uint8_t)tbytes};
    mb_write(&m, lb, 4);
    mb_write(&m, tb, tbytes);
    free(tb);

    /* pass 2: compress_to_writer (:177-227) */
    uint64_t maxbits = 0;
    {
        uint8_t* codes = (uint8_t*)calloc(256, CODE_STRIDE);
        uint32_t lens[256];
        uint32_t ml = orc_tree_codes(t, 256, codes, CODE_STRIDE, lens);
        free(codes);
        maxbits = (uint64_t)ml * (block_size < n ? block_size : n) + 8;
    }
    size_t blk_cap = (size_t)(maxbits / 8) + 16;
    uint8_t* comp = (uint8_t*)malloc(blk_cap);
    uint8_t* shifted = (uint8_t*)malloc(blk_cap + 8);
    uint8_t prev_byte = 0, prev_padding = 0;
    left = n; off = 0;
    for (;;) {
        /* `while reader.read_exact(buf).is_ok()` then `if left > 0` (tail) */
        size_t len;
        if (left >= block_size) len = block_size;
        else if (left > 0) len = left;
        else break;
        size_t clen;
        uint8_t pad, miss;
        int e = orc_compress_with_tree(file + off, len, t, comp, blk_cap, &clen, &pad, &miss);
        if (e) { free(comp); free(shifted); free(m.d); orc_tree_free(t); return e; }
        uint8_t* wbuf = comp;
        size_t wlen = clen;
        if (prev_padding != 0) {                        /* :196-201 */
            m.pos -= 1;                                 /* seek(Current(-1)) */
            wlen = orc_offset_bytes(comp, clen, prev_padding, shifted);
            shifted[0] |= prev_byte;
            wbuf = shifted;
        }
        mb_write(&m, wbuf, wlen);
        prev_padding = pad;                             /* :211 / :222 */
        prev_byte = wbuf[wlen - 1];                     /* :212 */
        off += len;
        left -= len;
        if (len < block_size) break;                    /* the tail is last */
    }
    free(comp);
    free(shifted);
    orc_tree_free(t);
    m.d[0] = (uint8_t)((tpad << 4) + prev_padding);     /* :69-70 */
    *out_len = m.len;
    if (out && cap >= m.len) memcpy(out, m.d, m.len);
    int rc = (out && cap >= m.len) || !out ? ORC_OK : ORC_E_BUFFER;
    free(m.d);
    return rc;
}

/* huff/src/comp.rs:79-157 read_decompress_write + :232-280 decompress_to_writer */
int orc_cli_decompress(const uint8_t* hff, size_t n, size_t block_size,
                       uint8_t* out, size_t cap, size_t* out_len)
{
    *out_len = 0;
    /* take(5).read(&mut buf): at most min(5, block_size) bytes */
    size_t first = n < 5 ? n : 5;
    if (first > block_size) first = block_size;
    if (first < 5) return ORC_E_MISSING_HEADER;                       /* :95-100 */
    uint8_t tpad = hff[0] >> 4, dpad = hff[0] & 0x0F;
    if (tpad > 7 || dpad > 7) return ORC_E_INVALID_HEADER;            /* :107-112 */
    size_t tlen = ((size_t)hff[1] << 24) | ((size_t)hff[2] << 16) | ((size_t)hff[3] << 8) | hff[4];
    size_t avail = n - 5;
    size_t got = tlen < avail ? tlen : avail;
    if (got > block_size) got = block_size;
    if (got < tlen) return ORC_E_MISSING_HEADER;                      /* :123-128 */
    size_t nbits = tlen * 8;
    uint8_t* bits = (uint8_t*)malloc(nbits + 1);
    for (size_t i = 0; i < nbits; ++i) bits[i] = (hff[5 + i / 8] >> (7 - i % 8)) & 1;
    nbits = tpad > nbits ? 0 : nbits - tpad;
    orc_tree* t = NULL;
    const char* msg;
    int e = orc_tree_try_from_bin(bits, nbits, 8, &t, &msg);
    free(bits);
    if (e) return ORC_E_INVALID_HEADER;                               /* :141-144 */

    const uint8_t* data = hff + 5 + tlen;
    size_t left = n - 5 - tlen, off = 0;
    walk_state s = {t, t->root, out, out ? cap : 0, 0};
    while (left >= block_size) {                                      /* :262-269 */
        for (size_t i = 0; i < block_size; ++i) walk_bits(&s, data[off + i], 8);
        off += block_size;
        left -= block_size;
    }
    if (left > 0) {                                                   /* :272-278 */
        for (size_t i = 0; i + 1 < left; ++i) walk_bits(&s, data[off + i], 8);
        walk_bits(&s, data[off + left - 1], 8 - dpad);
    }
    orc_tree_free(t);
    *out_len = s.count;
    return (out && s.count > cap) ? ORC_E_BUFFER : ORC_OK;
}

/* ======================================================================== */
/* table-driven checker                                                      */
/* ======================================================================== */

typedef struct {
    const uint8_t* in;
    size_t lo, hi;
    const uint64_t* code;
    const uint8_t* len;
    uint64_t bits;        /* phase 1 result */
    uint64_t start_bit;   /* absolute start bit (phase 2 input) */
    uint8_t* out;
    uint8_t* head;        /* private copy of the first (shared) byte */
    int phase;
} fast_job;

static void* fast_worker(void* p)
{
    fast_job* j = (fast_job*)p;
    if (j->phase == 1) {
        uint64_t b = 0;
        for (size_t i = j->lo; i < j->hi; ++i) b += j->len[j->in[i]];
        j->bits = b;
        return NULL;
    }
    /* phase 2: write bytes [start/8, end/8) except the first byte, which is
     * kept in head (OR-merged by the caller); the final partial byte too. */
    uint64_t pos = j->start_bit;
    uint64_t first_byte = pos / 8;
    unsigned __int128 acc = 0;
    unsigned nacc = (unsigned)(pos % 8);
    uint64_t wbyte = first_byte;
    *j->head = 0;
    for (size_t i = j->lo; i < j->hi; ++i) {
        uint8_t l = j->len[j->in[i]];
        acc = (acc << l) | j->code[j->in[i]];
        nacc += l;
        if (nacc >= 64) { /* 8 whole bytes, big-endian */
            uint64_t v = (uint64_t)(acc >> (nacc - 64));
            nacc -= 64;
            if (wbyte == first_byte) {
                *j->head = (uint8_t)(v >> 56);
                for (int k = 1; k < 8; ++k) j->out[wbyte + k] = (uint8_t)(v >> (56 - 8 * k));
            } else {
                v = __builtin_bswap64(v);
                memcpy(j->out + wbyte, &v, 8);
            }
            wbyte += 8;
        }
    }
    while (nacc >= 8) {
        uint8_t v = (uint8_t)(acc >> (nacc - 8));
        if (wbyte == first_byte) *j->head = v; else j->out[wbyte] = v;
        wbyte++;
        nacc -= 8;
    }
    if (nacc > 0) {
        uint8_t v = (uint8_t)(acc << (8 - nacc));
        if (wbyte == first_byte) *j->head |= v; else j->out[wbyte] = v;
    }
    return NULL;
}

int orc_fast_encode(const uint8_t* in, size_t n, const uint64_t code[256],
                    const uint8_t len[256], int threads, uint64_t bit_base,
                    uint8_t* out, size_t cap, uint64_t* total_bits)
{
    return orc_fast_encode_idx(in, n, code, len, threads, bit_base, out, cap, total_bits, NULL);
}

int orc_fast_encode_idx(const uint8_t* in, size_t n, const uint64_t code[256],
                        const uint8_t len[256], int threads, uint64_t bit_base,
                        uint8_t* out, size_t cap, uint64_t* total_bits, uint64_t* job_start)
{
    if (threads < 1) threads = 1;
    if ((size_t)threads > n / 4096 + 1) threads = (int)(n / 4096 + 1);
    fast_job* jobs = (fast_job*)calloc((size_t)threads, sizeof(fast_job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    uint8_t* heads = (uint8_t*)calloc((size_t)threads, 1);
    size_t per = n / (size_t)threads;
    for (int i = 0; i < threads; ++i) {
        jobs[i].in = in; jobs[i].code = code; jobs[i].len = len;
        jobs[i].lo = per * (size_t)i;
        jobs[i].hi = (i == threads - 1) ? n : per * (size_t)(i + 1);
        jobs[i].phase = 1;
        pthread_create(&th[i], NULL, fast_worker, &jobs[i]);
    }
    for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
    uint64_t pos = bit_base;
    for (int i = 0; i < threads; ++i) { jobs[i].start_bit = pos; pos += jobs[i].bits; }
    *total_bits = pos - bit_base;
    if (job_start)
        for (int i = 0; i < threads; ++i) job_start[i] = jobs[i].start_bit;
    size_t need = (size_t)((pos + 7) / 8);
    if (need > cap) { free(jobs); free(th); free(heads); return ORC_E_BUFFER; }
    /* every byte from bit_base/8 .. need is written by exactly one job or merged */
    for (int i = 0; i < threads; ++i) {
        jobs[i].phase = 2; jobs[i].out = out; jobs[i].head = &heads[i];
        pthread_create(&th[i], NULL, fast_worker, &jobs[i]);
    }
    for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
    /* first byte of job 0 ORs with whatever the caller already has there */
    for (int i = 0; i < threads; ++i) {
        uint64_t fb = jobs[i].start_bit / 8;
        if (jobs[i].bits == 0) continue;
        /* a partial first byte ORs with the bits the previous job (or the
         * caller, for job 0) already placed there; merged in job order */
        out[fb] = (uint8_t)((jobs[i].start_bit % 8 ? out[fb] : 0) | heads[i]);
    }
    free(jobs); free(th); free(heads);
    return ORC_OK;
}

typedef struct { const uint8_t* in; size_t lo, hi; uint64_t w[256]; } hist_job;

static void* hist_worker(void* p)
{
    hist_job* j = (hist_job*)p;
    memset(j->w, 0, sizeof(j->w));
    for (size_t i = j->lo; i < j->hi; ++i) j->w[j->in[i]]++;
    return NULL;
}

/* table-driven decode over the encoder's job partition: job i decodes the
 * letters [lo_i, hi_i) (split as in orc_fast_encode_idx) from bit start[i].
 * A 2^12-entry table resolves codes of <= 12 bits in one step; longer codes
 * continue bit by bit from the node the table reached. */
#define FAST_K 12
#define FAST_LEAF 0x80000000u

typedef struct {
    const uint8_t* comp;
    size_t comp_bytes;
    const orc_tree* t;
    const uint32_t* lut;
    size_t lo, hi;
    uint64_t start;
    uint8_t* out;
} fdec_job;

static inline uint64_t peek64(const uint8_t* comp, size_t nbytes, uint64_t bit)
{
    uint64_t byte = bit >> 3, v = 0;
    unsigned sh0 = (unsigned)(bit & 7);
    if (byte + 9 <= nbytes) {
        memcpy(&v, comp + byte, 8);
        v = __builtin_bswap64(v);
        return sh0 ? (v << sh0) | (comp[byte + 8] >> (8 - sh0)) : v;
    }
    for (int k = 0; k < 8; ++k) v = (v << 8) | (byte + k < nbytes ? comp[byte + k] : 0);
    unsigned sh = (unsigned)(bit & 7);
    uint64_t nx = byte + 8 < nbytes ? comp[byte + 8] : 0;
    return sh ? (v << sh) | (nx >> (8 - sh)) : v;
}

static void* fdec_worker(void* p)
{
    fdec_job* j = (fdec_job*)p;
    const orc_node* nd = j->t->nodes;
    uint64_t pos = j->start;
    for (size_t i = j->lo; i < j->hi; ++i) {
        uint64_t w = peek64(j->comp, j->comp_bytes, pos);
        uint32_t e = j->lut[w >> (64 - FAST_K)];
        if (e & FAST_LEAF) {
            j->out[i] = (uint8_t)e;
            pos += (e >> 8) & 0xFF;
            continue;
        }
        int32_t cur = (int32_t)e;
        pos += FAST_K;
        while (!nd[cur].leaf) {
            uint64_t bit = (j->comp[pos >> 3] >> (7 - (pos & 7))) & 1;
            cur = bit ? nd[cur].right : nd[cur].left;
            pos++;
        }
        j->out[i] = (uint8_t)nd[cur].letter;
    }
    return NULL;
}

int orc_fast_decode(const uint8_t* comp, size_t comp_bytes, const orc_tree* t, size_t n,
                    int threads, const uint64_t* job_start, uint8_t* out)
{
    if (threads < 1) threads = 1;
    if ((size_t)threads > n / 4096 + 1) threads = (int)(n / 4096 + 1);
    uint32_t* lut = (uint32_t*)malloc(sizeof(uint32_t) << FAST_K);
    const orc_node* nd = t->nodes;
    for (uint32_t p = 0; p < (1u << FAST_K); ++p) {
        int32_t cur = t->root;
        uint32_t d = 0;
        if (nd[cur].leaf) { /* single-leaf tree: one letter per bit */
            lut[p] = FAST_LEAF | (1u << 8) | (uint32_t)(uint8_t)nd[cur].letter;
            continue;
        }
        while (!nd[cur].leaf && d < FAST_K) {
            cur = ((p >> (FAST_K - 1 - d)) & 1) ? nd[cur].right : nd[cur].left;
            d++;
        }
        lut[p] = nd[cur].leaf ? FAST_LEAF | (d << 8) | (uint32_t)(uint8_t)nd[cur].letter : (uint32_t)cur;
    }
    fdec_job* jobs = (fdec_job*)calloc((size_t)threads, sizeof(fdec_job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    size_t per = n / (size_t)threads;
    for (int i = 0; i < threads; ++i) {
        fdec_job* j = &jobs[i];
        j->comp = comp; j->comp_bytes = comp_bytes; j->t = t; j->lut = lut; j->out = out;
        j->lo = per * (size_t)i;
        j->hi = (i == threads - 1) ? n : per * (size_t)(i + 1);
        j->start = job_start[i];
        pthread_create(&th[i], NULL, fdec_worker, j);
    }
    for (int i = 0; i < threads; ++i) pthread_join(th[i], NULL);
    free(jobs); free(th); free(lut);
    return ORC_OK;
}

void orc_fast_hist(const uint8_t* in, size_t n, int threads, uint64_t w[256])
{
    if (threads < 1) threads = 1;
    hist_job* jobs = (hist_job*)calloc((size_t)threads, sizeof(hist_job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    size_t per = n / (size_t)threads;
    for (int i = 0; i < threads; ++i) {
        jobs[i].in = in;
        jobs[i].lo = per * (size_t)i;
        jobs[i].hi = (i == threads - 1) ? n : per * (size_t)(i + 1);
        pthread_create(&th[i], NULL, hist_worker, &jobs[i]);
    }
    memset(w, 0, 256 * sizeof(uint64_t));
    for (int i = 0; i < threads; ++i) {
        pthread_join(th[i], NULL);
        for (int b = 0; b < 256; ++b) w[b] += jobs[i].w[b];
    }
    free(jobs); free(th);
}

/* ======================================================================== */
/* synthetic inputs — counter-based, reproduced by the product's generator    */
/* ======================================================================== */

/* splitmix64: output k of the stream seeded with `seed` */
uint64_t orc_splitmix64(uint64_t k, uint64_t seed)
{
    uint64_t z = seed + (k + 1) * 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

/* byte i = little-endian byte (i % 8) of output (i / 8) */
void orc_gen_uniform(uint64_t seed, uint64_t offset, size_t n, uint8_t* out)
{
    for (size_t i = 0; i < n; ++i) {
        uint64_t g = offset + i;
        out[i] = (uint8_t)(orc_splitmix64(g / 8, seed) >> (8 * (g % 8)));
    }
}

/* P(rank k) ~ k^-alpha, k = 1..256, byte = k-1; cdf[k-1] = floor(2^64 * P(<=k)),
 * cdf[255] = UINT64_MAX. The table is an INPUT of the device generator. */
void orc_zipf_cdf(double alpha, uint64_t cdf[256])
{
    double p[256], s = 0;
    for (int k = 1; k <= 256; ++k) {
        double v = pow((double)k, -alpha);
        p[k - 1] = v;
        s += v;
    }
    double acc = 0;
    for (int k = 0; k < 256; ++k) {
        acc += p[k] / s;
        double scaled = acc * 18446744073709551616.0;
        cdf[k] = (scaled >= 18446744073709551615.0) ? UINT64_MAX : (uint64_t)scaled;
    }
    cdf[255] = UINT64_MAX;
}

static uint8_t zipf_pick(uint64_t r, const uint64_t cdf[256])
{
    /* first k with r < cdf[k] (cdf[255] = max catches the rest) */
    int lo = 0, hi = 255;
    while (lo < hi) {
        int mid = (lo + hi) / 2;
        if (r < cdf[mid]) hi = mid; else lo = mid + 1;
    }
    return (uint8_t)lo;
}

void orc_gen_zipf(uint64_t seed, uint64_t offset, size_t n, const uint64_t cdf[256], uint8_t* out)
{
    for (size_t i = 0; i < n; ++i) out[i] = zipf_pick(orc_splitmix64(offset + i, seed), cdf);
}

/* Deterministic English-like text, 64-byte lines: words drawn with a skew
 * from a 512-word synthetic vocabulary, separated by spaces, '\n' at byte 63.
 * Line l depends only on (seed, l), so the device generates it identically. */
static void gen_word(uint32_t k, uint8_t* w, int* len)
{
    uint64_t h = orc_splitmix64(k, 0x7E47ULL);
    int l = 1 + (int)(h % 9);
    static const char letters[] = "etaoinshrdlucmfwypvbgkjqxz";
    for (int i = 0; i < l; ++i) {
        uint64_t r = (h >> (6 + 5 * (i % 10))) ^ (uint64_t)i * 0x9E37ULL;
        /* skew toward frequent letters: min of two draws */
        int a = (int)(r % 26), b = (int)((r >> 7) % 26);
        w[i] = (uint8_t)letters[a < b ? a : b];
    }
    *len = l;
}

void orc_gen_text(uint64_t seed, uint64_t offset, size_t n, uint8_t* out)
{
    uint8_t line[64];
    uint64_t cur_line = UINT64_MAX;
    for (size_t i = 0; i < n; ++i) {
        uint64_t g = offset + i;
        uint64_t l = g / 64;
        if (l != cur_line) {
            cur_line = l;
            int p = 0;
            uint64_t st = 0;
            while (p < 63) {
                uint64_t r = orc_splitmix64(l * 16 + st++, seed);
                uint32_t span = (uint32_t)(r & 511) + 1;
                uint32_t k = (uint32_t)((r >> 9) % span);
                uint8_t w[10];
                int wl;
                gen_word(k, w, &wl);
                for (int q = 0; q < wl && p < 63; ++q) line[p++] = w[q];
                if (p < 63) line[p++] = (r >> 40) % 11 == 0 ? ',' : ' ';
                if (st >= 16) { while (p < 63) line[p++] = ' '; }
            }
            line[63] = '\n';
        }
        out[i] = line[g % 64];
    }
}

double orc_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}
