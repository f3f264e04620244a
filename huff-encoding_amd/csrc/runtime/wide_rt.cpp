// wide_rt.cpp — the wider-letter job and host-pointer pipelines
// (wide_rt.hpp; kernels in device/wide.hip, device/wweights.hip).
#include "wide_rt.hpp"

#include <atomic>
#include <cstring>

namespace {
std::atomic<uint64_t> g_wtree_ids{1};
constexpr size_t kTableLdsMax = 64 * 1024;  // stage the code hash table in LDS up to this
}  // namespace

#define HIP_TRY(expr) HIP_TRY_RT(expr)

using huff::Status;

huff_wtree::huff_wtree() : id(g_wtree_ids.fetch_add(1)) {}

Status huff_wtree::enc_tables(const huff::WideEncTables** out) const {
    std::lock_guard<std::mutex> g(m);
    if (!enc) {
        auto e = std::make_unique<huff::WideEncTables>();
        HUFF_TRY(huff::build_wide_enc_tables(t, *e));
        enc = std::move(e);
    }
    *out = enc.get();
    return Status::ok();
}

Status huff_wtree::dec_tables(const huff::WideDecTables** out) const {
    std::lock_guard<std::mutex> g(m);
    if (!dec) {
        auto d = std::make_unique<huff::WideDecTables>();
        HUFF_TRY(huff::build_wide_dec_tables(t, *d));
        dec = std::move(d);
    }
    *out = dec.get();
    return Status::ok();
}

const huff_tree* huff_wtree::shape_tree() const {
    std::lock_guard<std::mutex> g(m);
    if (!shape) {
        shape = std::make_unique<huff_tree>();
        shape->t = t.shape();
    }
    return shape.get();
}

// ---------------------------------------------------------------------------
Status huff_wenc::init(huff_ctx* c, uint32_t w, const uint8_t* d, uint64_t nletters) {
    if (!huff::valid_width(w)) return Status::err(HUFF_E_INVALID_ARG, "letter width must be 1, 2, 4, 8 or 16 bytes");
    if (reinterpret_cast<uintptr_t>(d) & 15) return Status::err(HUFF_E_INVALID_ARG, "letters must be 16-byte aligned");
    if (nletters >= (uint64_t(1) << 44)) return Status::err(HUFF_E_INVALID_ARG, "too many letters for one job");
    ctx = c;
    width = w;
    d_in = d;
    n = nletters;
    nchunks = static_cast<uint32_t>((n + huff::dev::kWideChunk - 1) / huff::dev::kWideChunk);
    HUFF_TRY(chunk_bits.ensure((nchunks + 1) * 8));
    HUFF_TRY(chunk_start.ensure((nchunks + 2) * 8));
    HUFF_TRY(tsum.ensure((nchunks / 1024 + 2) * 8));
    HUFF_TRY(sub_bit.ensure(((n + huff::dev::kWideRun - 1) / huff::dev::kWideRun + 1) * 4));
    HUFF_TRY(missing.ensure(8));
    return Status::ok();
}

huff::dev::WideArgs huff_wenc::enc_args(bool pack_pass) const {
    huff::dev::WideArgs a{};
    a.in = d_in;
    a.n = n;
    a.width = width;
    a.table = table.p;
    a.slots = et->slots;
    a.slot_bytes = et->slot_bytes;
    a.mul1 = et->mul1;
    a.hash_mode = et->hash_mode;
    a.fold = et->fold;
    a.long_codes = et->long_codes;
    a.max_len = et->maxlen;
    a.nchunks = nchunks;
    a.cu_count = static_cast<uint32_t>(ctx->cu_count);
    a.stage_words = huff::dev::wide_stage_words(width, et->maxlen);
    a.table_in_lds = huff::dev::wide_lds_bytes(a, pack_pass, true) <= huff::dev::kWideLdsMax;
    return a;
}

Status huff_wenc::bits(const huff_wtree* t, uint64_t* total, huff::u128* missing_letter) {
    HUFF_TRY(ctx->activate());
    HUFF_TRY(t->enc_tables(&et));
    if (et->width != width) return Status::err(HUFF_E_INVALID_ARG, "the tree's letter width differs from the job's");
    hipStream_t s = ctx->stream;
    if (enc_tree != t->id) {
        HUFF_TRY(table.ensure(et->table.size()));
        HIP_TRY(hipMemcpyAsync(table.p, et->table.data(), et->table.size(), hipMemcpyHostToDevice, s));
        enc_tree = t->id;
    }
    HIP_TRY(hipMemsetAsync(missing.p, 0xFF, 8, s));
    huff::dev::WideArgs a = enc_args(false);
    a.chunk_bits = static_cast<uint64_t*>(chunk_bits.p);
    a.sub_bit = static_cast<uint32_t*>(sub_bit.p);
    a.first_missing = static_cast<unsigned long long*>(missing.p);
    HUFF_TRY(ctx->timed("wbits", [&] { return huff::dev::launch_wide_bits(a, s); }));
    HUFF_TRY(ctx->timed("wscan", [&] {
        return huff::dev::launch_scan(static_cast<const uint64_t*>(chunk_bits.p), nchunks, 0,
                                      static_cast<uint64_t*>(chunk_start.p), static_cast<uint64_t*>(tsum.p), s);
    }));
    uint64_t hv[2] = {0, 0};
    HIP_TRY(hipMemcpyAsync(&hv[0], static_cast<uint64_t*>(chunk_start.p) + nchunks, 8, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(&hv[1], missing.p, 8, hipMemcpyDeviceToHost, s));
    HUFF_TRY(ctx->sync());
    bits_tree = 0;
    if (hv[1] != ~0ull) {  // comp.rs:426-432: the first letter (input order) with no code
        uint8_t lb[16] = {};
        HIP_TRY(hipMemcpy(lb, d_in + hv[1] * width, width, hipMemcpyDeviceToHost));
        if (missing_letter) *missing_letter = huff::load_letter(lb, width);
        return Status::err(HUFF_E_MISSING_LETTER, "letter not found in codes");
    }
    total_bits = hv[0];
    bits_tree = t->id;
    if (total) *total = total_bits;
    return Status::ok();
}

Status huff_wenc::pack(const huff_wtree* t, uint8_t* d_out, size_t out_cap, uint64_t* total) {
    if (bits_tree != t->id) HUFF_TRY(bits(t, nullptr, nullptr));
    if (total) *total = total_bits;
    const uint64_t need = (total_bits + 7) / 8;
    if (out_cap < need) return Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
    huff::dev::WideArgs a = enc_args(true);
    a.chunk_start = static_cast<const uint64_t*>(chunk_start.p);
    a.out = d_out;
    hipStream_t s = ctx->stream;
    return ctx->timed("wpack", [&] { return huff::dev::launch_wide_pack(a, s); });
}

Status huff_wenc::upload_dec(const huff_wtree* t) {
    HUFF_TRY(t->dec_tables(&dt));
    if (t->t.width() != width) return Status::err(HUFF_E_INVALID_ARG, "the tree's letter width differs from the job's");
    if (dec_tree == t->id) return Status::ok();
    HUFF_TRY(lut.ensure(dt->lut.size() * 4));
    HUFF_TRY(letters.ensure((dt->letters.size() + 31) / 16 * 16));  // staged in 16-B pieces
    HUFF_TRY(stab.ensure(dt->stab.size()));
    HIP_TRY(hipMemcpyAsync(lut.p, dt->lut.data(), dt->lut.size() * 4, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(letters.p, dt->letters.data(), dt->letters.size(), hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(hipMemcpyAsync(stab.p, dt->stab.data(), dt->stab.size(), hipMemcpyHostToDevice, ctx->stream));
    dec_tree = t->id;
    return Status::ok();
}

Status huff_wenc::decode(const huff_wtree* t, const uint8_t* d_comp, uint64_t comp_bytes, uint8_t* d_out,
                         const uint64_t* sub_abs, bool skip_packed) {
    HUFF_TRY(ctx->activate());
    if (reinterpret_cast<uintptr_t>(d_comp) & 15) {
        // the decoders read the stream in dwords and 16-B pieces: a stream at
        // any other alignment (packed into a tensor view at an odd offset,
        // which huff_wenc_pack allows) is copied once to an aligned buffer
        HUFF_TRY(ctx->d_comp_align.ensure(comp_bytes + 64));
        HIP_TRY(hipMemcpyAsync(ctx->d_comp_align.p, d_comp, comp_bytes, hipMemcpyDeviceToDevice, ctx->stream));
        d_comp = static_cast<const uint8_t*>(ctx->d_comp_align.p);
    }
    HUFF_TRY(upload_dec(t));
    huff::dev::WideDecArgs a{};
    a.comp = d_comp;
    a.comp_bytes = comp_bytes;
    a.lut = static_cast<const uint32_t*>(lut.p);
    a.lut_bits = dt->bits;
    a.stab = stab.p;
    a.stab_bits = dt->sbits;
    a.stab_bytes = static_cast<uint32_t>(dt->stab.size());
    a.letters = static_cast<const uint8_t*>(letters.p);
    a.nleaves = static_cast<uint32_t>(dt->letters.size() / width);
    a.w4_leaf = dt->w4_leaf ? 1u : 0u;
    a.max_len = dt->maxdepth;
    a.width = width;
    a.chunk_start = static_cast<const uint64_t*>(chunk_start.p);
    a.sub_bit = static_cast<const uint32_t*>(sub_bit.p);
    a.sub_abs = sub_abs;
    a.skip_packed = skip_packed ? 1u : 0u;
    a.nchunks = nchunks;
    a.cu_count = static_cast<uint32_t>(ctx->cu_count);
    a.n = n;
    a.out = d_out;
    a.end_bit = comp_bytes * 8;  // bounds the last task's staged range
    hipStream_t s = ctx->stream;
    if (!dt->stab.empty()) {
        // the task decoder's LDS stage per wave: the task's mean compressed
        // bytes with a quarter of headroom (tasks beyond it decode from
        // global memory), 2..16 KiB
        const double bits_per = n ? static_cast<double>(comp_bytes) * 8.0 / static_cast<double>(n) : 8.0;
        const double want = 1.25 * bits_per * huff::dev::kWideRun * 64 / 8 + 96;
        uint32_t sb = static_cast<uint32_t>(want < 2048 ? 2048 : (want > 16384 ? 16384 : want));
        a.stage_bytes = (sb + 15) & ~15u;
        return ctx->timed("wdecode", [&] { return huff::dev::launch_wide_decode_task(a, s); });
    }
    if (skip_packed) return Status::err(HUFF_E_INVALID_ARG, "skip marks need the task decoder (codes <= 32 bits)");
    return ctx->timed("wdecode", [&] { return huff::dev::launch_wide_decode(a, s); });
}

Status huff_wenc::download_index(huff_index_host& idx) {
    idx.n = n;
    idx.chunk_start.resize(nchunks + 1);
    idx.sub_bit.resize((n + huff::dev::kWideRun - 1) / huff::dev::kWideRun);
    HIP_TRY(hipMemcpyAsync(idx.chunk_start.data(), chunk_start.p, idx.chunk_start.size() * 8, hipMemcpyDeviceToHost,
                           ctx->stream));
    if (!idx.sub_bit.empty())
        HIP_TRY(hipMemcpyAsync(idx.sub_bit.data(), sub_bit.p, idx.sub_bit.size() * 4, hipMemcpyDeviceToHost,
                               ctx->stream));
    return ctx->sync();
}

Status huff_wenc::upload_index(const huff_index_host& idx) {
    if (idx.n != n || idx.chunk_start.size() != nchunks + 1u)
        return Status::err(HUFF_E_INVALID_ARG, "restart index does not match the job");
    HIP_TRY(hipMemcpyAsync(chunk_start.p, idx.chunk_start.data(), idx.chunk_start.size() * 8, hipMemcpyHostToDevice,
                           ctx->stream));
    if (!idx.sub_bit.empty())
        HIP_TRY(hipMemcpyAsync(sub_bit.p, idx.sub_bit.data(), idx.sub_bit.size() * 4, hipMemcpyHostToDevice,
                               ctx->stream));
    return Status::ok();
}

// ---------------------------------------------------------------------------
namespace huff {

Status wweights_map_host(huff_ctx* ctx, uint32_t width, const uint8_t* letters, size_t n,
                         std::vector<uint8_t>& uniq, std::vector<uint64_t>& counts) {
    // build_weights_map (weights.rs:82-123) on the device (wweights.hip),
    // distinct letters in ascending order
    uniq.clear();
    counts.clear();
    if (!valid_width(width)) return Status::err(HUFF_E_INVALID_ARG, "letter width must be 1, 2, 4, 8 or 16 bytes");
    if (n == 0) return Status::ok();
    HUFF_TRY(ctx->activate());
    hipStream_t s = ctx->stream;
    const size_t nb = n * width;
    HUFF_TRY(ctx->d_in.ensure(nb + 16));
    HIP_TRY(hipMemcpyAsync(ctx->d_in.p, letters, nb, hipMemcpyHostToDevice, s));
    dev::WCountArgs a{};
    a.in = static_cast<const uint8_t*>(ctx->d_in.p);
    a.n = n;
    a.width = width;
    const auto put = [&](uint64_t lo, uint64_t hi, uint64_t c) {
        for (uint32_t j = 0; j < width; ++j) uniq.push_back(static_cast<uint8_t>(j < 8 ? lo >> (8 * j) : hi >> (8 * (j - 8))));
        counts.push_back(c);
    };
    DevBuf cnt, klo, khi, state, olo, ohi, oc, misc;
    if (width <= 2) {  // direct bins: ascending by construction
        a.slots = dev::wcount_slots(width, n);
        HUFF_TRY(cnt.ensure(a.slots * 8));
        HIP_TRY(hipMemsetAsync(cnt.p, 0, a.slots * 8, s));
        a.counts = static_cast<unsigned long long*>(cnt.p);
        HUFF_TRY(ctx->timed("wweights", [&] { return dev::wcount_launch(a, s); }));
        std::vector<uint64_t> bins(a.slots);
        HIP_TRY(hipMemcpyAsync(bins.data(), cnt.p, a.slots * 8, hipMemcpyDeviceToHost, s));
        HUFF_TRY(ctx->sync());
        for (uint64_t k = 0; k < a.slots; ++k)
            if (bins[k]) put(k, 0, bins[k]);
        return Status::ok();
    }
    // the HBM table sized for a guess of the distinct letters (at most 2^19,
    // 8 MiB of slots for W = 4 / 8) and grown when the kernel reports it too
    // full: ~16-32 B per slot, so a table for n distinct letters of a 1 GiB
    // input would be ~12x the input where a few thousand letters are the
    // common case. The largest size (2 n slots) counts without limits.
    const uint64_t max_slots = dev::wcount_slots(width, n);
    a.slots = std::min(max_slots, dev::wcount_slots(width, std::min<uint64_t>(n, 1ull << 19)));
    HUFF_TRY(misc.ensure(32));
    uint64_t m[4] = {};  // nout, sent, used, overflow
    for (;;) {
        a.unbounded = a.slots >= max_slots ? 1u : 0u;
        HUFF_TRY(cnt.ensure(a.slots * 8));
        HIP_TRY(hipMemsetAsync(cnt.p, 0, a.slots * 8, s));
        a.counts = static_cast<unsigned long long*>(cnt.p);
        HUFF_TRY(klo.ensure(a.slots * 8));
        HIP_TRY(hipMemsetAsync(klo.p, 0xFF, a.slots * 8, s));
        a.keys_lo = static_cast<unsigned long long*>(klo.p);
        if (width == 16) {
            HUFF_TRY(khi.ensure(a.slots * 8));
            HUFF_TRY(state.ensure(a.slots * 4));
            HIP_TRY(hipMemsetAsync(state.p, 0, a.slots * 4, s));
            a.keys_hi = static_cast<unsigned long long*>(khi.p);
            a.state = static_cast<unsigned int*>(state.p);
        }
        HIP_TRY(hipMemsetAsync(misc.p, 0, 32, s));
        a.nout = static_cast<unsigned long long*>(misc.p);
        a.sent = a.nout + 1;
        a.used = a.nout + 2;
        a.overflow = reinterpret_cast<unsigned int*>(a.nout + 3);
        HUFF_TRY(ctx->timed("wweights", [&] { return dev::wcount_launch(a, s); }));
        HIP_TRY(hipMemcpyAsync(m, misc.p, 32, hipMemcpyDeviceToHost, s));
        HUFF_TRY(ctx->sync());
        if (!(m[3] & 1) || a.unbounded) break;
        // at least m[2] distinct letters: room for twice as many, or 4x the slots
        a.slots = std::min(max_slots, std::max(a.slots * 4, dev::wcount_slots(width, 2 * m[2])));
    }
    // the outputs hold the claimed slots only
    const uint64_t cap = std::max<uint64_t>(m[2], 1);
    HUFF_TRY(olo.ensure(cap * 8));
    HUFF_TRY(oc.ensure(cap * 8));
    if (width == 16) HUFF_TRY(ohi.ensure(cap * 8));
    a.out_lo = static_cast<unsigned long long*>(olo.p);
    a.out_c = static_cast<unsigned long long*>(oc.p);
    a.out_hi = width == 16 ? static_cast<unsigned long long*>(ohi.p) : nullptr;
    a.out_cap = cap;  // a guard the kernel enforces, so the check below comes before any overrun
    HIP_TRY(dev::wextract_launch(a, s));
    HIP_TRY(hipMemcpyAsync(m, misc.p, 8, hipMemcpyDeviceToHost, s));
    HUFF_TRY(ctx->sync());
    if (m[0] > cap) return Status::err(HUFF_E_HIP, "wide weights: more used slots than claims");
    std::vector<uint64_t> lo(m[0]), hi(width == 16 ? m[0] : 0), c(m[0]);
    if (m[0]) {
        HIP_TRY(hipMemcpyAsync(lo.data(), olo.p, m[0] * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(c.data(), oc.p, m[0] * 8, hipMemcpyDeviceToHost, s));
        if (width == 16) HIP_TRY(hipMemcpyAsync(hi.data(), ohi.p, m[0] * 8, hipMemcpyDeviceToHost, s));
        HUFF_TRY(ctx->sync());
    }
    std::vector<uint64_t> order(m[0]);
    for (uint64_t i = 0; i < m[0]; ++i) order[i] = i;
    std::sort(order.begin(), order.end(), [&](uint64_t x, uint64_t y) {
        if (width == 16 && hi[x] != hi[y]) return hi[x] < hi[y];
        return lo[x] < lo[y];
    });
    for (uint64_t i : order) put(lo[i], width == 16 ? hi[i] : 0, c[i]);
    if (m[1]) put(~0ull, 0, m[1]);  // the all-ones u64 letter (the table's empty marker) sorts last
    return Status::ok();
}

Status wcompress_host(huff_ctx* ctx, uint32_t width, const uint8_t* letters, size_t n, const huff_wtree* t,
                      huff_wcompress_data** out, u128* missing) {
    *out = nullptr;
    std::unique_ptr<huff_wtree> own;
    if (!t) {  // compress (comp.rs:353-359): the tree of build_weights_map
        std::vector<uint8_t> uniq;
        std::vector<uint64_t> counts;
        HUFF_TRY(wweights_map_host(ctx, width, letters, n, uniq, counts));
        own = std::make_unique<huff_wtree>();
        HUFF_TRY(WideTree::from_weights(width, uniq.data(), counts.data(), counts.size(), own->t));
        t = own.get();
    }
    if (t->t.width() != width) return Status::err(HUFF_E_INVALID_ARG, "the tree's letter width differs from the letters'");
    // comp.rs:443-449: no letters -> no bytes -> CompressData::new panics
    if (n == 0) return Status::err(HUFF_E_EMPTY_COMP, "provided comp_bytes are empty");
    HUFF_TRY(ctx->activate());
    hipStream_t s = ctx->stream;
    HUFF_TRY(ctx->d_in.ensure(n * width + 16));
    HIP_TRY(hipMemcpyAsync(ctx->d_in.p, letters, n * width, hipMemcpyHostToDevice, s));
    huff_wenc e;
    HUFF_TRY(e.init(ctx, width, static_cast<const uint8_t*>(ctx->d_in.p), n));
    uint64_t tb = 0;
    HUFF_TRY(e.bits(t, &tb, missing));
    const size_t words = static_cast<size_t>((tb + 31) / 32);
    HUFF_TRY(ctx->d_out.ensure(words * 4 + 16));
    HUFF_TRY(e.pack(t, static_cast<uint8_t*>(ctx->d_out.p), words * 4, &tb));
    auto cd = std::make_unique<huff_wcompress_data>();
    cd->comp.resize(static_cast<size_t>((tb + 7) / 8));
    HIP_TRY(hipMemcpyAsync(cd->comp.data(), ctx->d_out.p, cd->comp.size(), hipMemcpyDeviceToHost, s));
    cd->padding = calc_padding_bits(tb);  // comp.rs:446
    cd->index = std::make_unique<huff_index_host>();
    HUFF_TRY(e.download_index(*cd->index));
    if (own) {
        cd->tree = own.release();
    } else {
        cd->tree = new huff_wtree();
        cd->tree->t = t->t;
    }
    *out = cd.release();
    return Status::ok();
}

Status wdecode_indexless_dev(huff_ctx* ctx, const huff_wtree* t, const uint8_t* d_comp, uint64_t comp_bytes,
                             uint64_t valid_bits, uint8_t* d_out, size_t cap_letters, uint64_t* n_out) {
    *n_out = 0;
    if (valid_bits == 0) return Status::ok();
    HUFF_TRY(ctx->activate());
    if (reinterpret_cast<uintptr_t>(d_comp) & 15) {  // the sync kernels stage 16-B pieces: an aligned copy
        HUFF_TRY(ctx->d_comp_align.ensure(comp_bytes + 64));
        HIP_TRY(hipMemcpyAsync(ctx->d_comp_align.p, d_comp, comp_bytes, hipMemcpyDeviceToDevice, ctx->stream));
        d_comp = static_cast<const uint8_t*>(ctx->d_comp_align.p);
    }
    // synchronise on the tree's shape (the sync kernels only use code lengths)
    const huff_tree* shape = t->shape_tree();
    const DecTables* dt = nullptr;
    HUFF_TRY(ctx->upload_dec_tables(shape, &dt));
    IndexlessSync& st = ctx->indexless_ws();
    st.dt = dt;
    const WideDecTables* wdt = nullptr;
    HUFF_TRY(t->dec_tables(&wdt));
    const bool skip = !wdt->stab.empty() && !std::getenv("HUFF_WIDE_MARK_WALK");
    DevBuf& sub_abs = ctx->idx_sub_abs;
    // every kWideRun-th letter: the task decoder (the tree's two-level table)
    // takes k_mark_lite's marks (a boundary and the codes to skip from it, as
    // the byte path's skip build), launched before the host waits for the
    // count (sized for the most letters the buffer or the stream holds);
    // HUFF_WIDE_MARK_WALK=1 or the long-code decoder: exact points walked by
    // k_mark_lds
    bool marked = false;
    auto mark_early = [&]() -> Status {
        if (!skip || !d_out || !st.block_off || !dev::indexless_staged(st.a)) return Status::ok();
        uint32_t min_len = 64, max_len_;
        shape->t.depth_range(&min_len, &max_len_);
        const uint64_t runs = (std::min<uint64_t>(cap_letters, valid_bits / min_len) + 63) >> 6;
        HUFF_TRY(sub_abs.ensure(runs * 8 + 8));
        HIP_TRY(dev::launch_indexless_mark_lite(st.a, nullptr, static_cast<const unsigned long long*>(st.woff.p),
                                                static_cast<uint64_t*>(sub_abs.p), runs, ctx->stream));
        marked = true;
        return Status::ok();
    };
    HUFF_TRY(indexless_sync(ctx, d_comp, comp_bytes, valid_bits, shape, st, !skip, mark_early));
    *n_out = st.total;
    if (!d_out) return Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
    if (st.total > cap_letters) return Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
    if (!dev::indexless_staged(st.a))
        return Status::err(HUFF_E_CODE_TOO_LONG, "index-free decode of letters wider than a byte needs codes <= 32 bits");
    if (skip && !marked) {
        HUFF_TRY(sub_abs.ensure(((st.total + 63) >> 6) * 8 + 8));
        HIP_TRY(dev::launch_indexless_mark_lite(
            st.a, st.block_off ? nullptr : static_cast<const uint64_t*>(st.off.p),
            st.block_off ? static_cast<const unsigned long long*>(st.woff.p) : nullptr,
            static_cast<uint64_t*>(sub_abs.p), ~0ull, ctx->stream));
    } else if (!skip) {
        HUFF_TRY(indexless_mark(ctx, st, sub_abs, 6));
    }
    HIP_TRY(hipEventRecord(ctx->lut_free, ctx->stream));
    // one task decoder per context: its buffers only grow and its tables
    // upload once per tree (a fresh one per call allocated and freed ~40 MB)
    if (!ctx->wdec_ws) ctx->wdec_ws = std::make_shared<huff_wenc>();
    huff_wenc& e = *ctx->wdec_ws;
    HUFF_TRY(e.init(ctx, t->t.width(), nullptr, st.total));
    HUFF_TRY(e.decode(t, d_comp, comp_bytes, d_out, static_cast<const uint64_t*>(sub_abs.p), skip));
    return ctx->sync();
}

Status wdecompress_host(huff_ctx* ctx, const huff_wcompress_data* cd, uint8_t* out, size_t cap_letters,
                        size_t* n_out) {
    const uint32_t W = cd->tree->t.width();
    HUFF_TRY(ctx->activate());
    hipStream_t s = ctx->stream;
    HUFF_TRY(ctx->d_in.ensure(cd->comp.size() + 16));
    HIP_TRY(hipMemcpyAsync(ctx->d_in.p, cd->comp.data(), cd->comp.size(), hipMemcpyHostToDevice, s));
    if (!cd->index) {
        // comp.rs:513-516: all bytes but the last give 8 bits, the last 8 - padding
        const uint64_t valid = static_cast<uint64_t>(cd->comp.size()) * 8 - cd->padding;
        uint64_t cnt = 0;
        Status q = wdecode_indexless_dev(ctx, cd->tree, static_cast<const uint8_t*>(ctx->d_in.p), cd->comp.size(),
                                         valid, nullptr, 0, &cnt);
        if (q.code != HUFF_E_BUFFER_TOO_SMALL && q.code != HUFF_OK) return q;
        *n_out = cnt;
        if (cap_letters < cnt) return Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
        if (cnt == 0) return Status::ok();
        HUFF_TRY(ctx->d_out.ensure(cnt * W + 16));
        HUFF_TRY(wdecode_indexless_dev(ctx, cd->tree, static_cast<const uint8_t*>(ctx->d_in.p), cd->comp.size(),
                                       valid, static_cast<uint8_t*>(ctx->d_out.p), cnt, &cnt));
        HIP_TRY(hipMemcpyAsync(out, ctx->d_out.p, cnt * W, hipMemcpyDeviceToHost, s));
        return ctx->sync();
    }
    const uint64_t n = cd->index->n;
    *n_out = n;
    if (cap_letters < n) return Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
    if (n == 0) return Status::ok();
    HUFF_TRY(ctx->d_out.ensure(n * W + 16));
    huff_wenc e;
    HUFF_TRY(e.init(ctx, W, nullptr, n));
    HUFF_TRY(e.upload_index(*cd->index));
    HUFF_TRY(e.decode(cd->tree, static_cast<const uint8_t*>(ctx->d_in.p), cd->comp.size(),
                      static_cast<uint8_t*>(ctx->d_out.p)));
    HIP_TRY(hipMemcpyAsync(out, ctx->d_out.p, n * W, hipMemcpyDeviceToHost, s));
    return ctx->sync();
}

}  // namespace huff
