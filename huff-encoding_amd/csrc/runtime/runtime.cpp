// runtime.cpp — context, encode job and host-pointer pipelines.
#include "runtime.hpp"

#include <algorithm>
#include <cmath>
#include <cctype>
#include <chrono>
#include <numeric>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>

namespace {

std::atomic<uint64_t> g_tree_ids{1};

}  // namespace

#define HIP_TRY(expr) HIP_TRY_RT(expr)

// ---------------------------------------------------------------------------
// trees and their tables
// ---------------------------------------------------------------------------
huff_tree::huff_tree() : id(g_tree_ids.fetch_add(1)) {}

const huff::EncTables& huff_tree::enc_tables() const {
    std::lock_guard<std::mutex> g(m);
    if (!enc) {
        auto e = std::make_unique<huff::EncTables>();
        e->fits64 = t.read_codes_u64(e->code, e->len, &e->maxlen);
        if (e->maxlen > huff::dev::kLongMaxLen) {  // deep codes: left-aligned words (deep.hip)
            std::array<std::vector<uint8_t>, 256> bits;
            t.read_codes(bits);
            e->deep.assign(256 * huff::dev::kDeepWords, 0);
            for (int b = 0; b < 256; ++b)
                for (size_t k = 0; k < bits[b].size(); ++k)
                    if (bits[b][k]) e->deep[b * huff::dev::kDeepWords + k / 32] |= 0x80000000u >> (k % 32);
        }
        enc = std::move(e);
    }
    return *enc;
}

huff::Status huff_tree::dec_tables(const huff::DecTables** out) const {
    std::lock_guard<std::mutex> g(m);
    if (!dec) {
        auto d = std::make_unique<huff::DecTables>();
        HUFF_TRY(huff::build_dec_tables(t, *d));
        dec = std::move(d);
    }
    *out = dec.get();
    return huff::Status::ok();
}

huff_compress_data::~huff_compress_data() { delete tree; }

namespace huff {

bool fixed8_disabled() {
    const char* e = std::getenv("HUFF_DISABLE_FIXED8");  // read per call: tests flip it
    return e && *e && *e != '0';
}

// HUFF_SMALL_STAGE=0: the decoders keep the 4.5 KiB stage for every stream (A/B)
bool small_stage_enabled() {
    const char* e = std::getenv("HUFF_SMALL_STAGE");  // read per call: tests flip it
    return !(e && *e == '0');
}

// HUFF_DMA_DECODE=1: the persistent LDS-DMA decoder (k_decode_dma; measured
// 8-15 % slower than the one-shot register-staged one, profiles/r06/decode_bound/)
uint32_t dma_decode_enabled() {
    const char* e = std::getenv("HUFF_DMA_DECODE");  // read per call: tests flip it
    return (e && *e == '1') ? 1u : 0u;
}

uint32_t decode_check_mode() {
    const char* e = std::getenv("HUFF_DEC_VARIANT");  // read per call: tests flip it
    if (!e) return 0;
    // 11: k_decode_fixed's self-checking build; every other value is the
    // production decoder (the round-2 diagnostics 12-14 are not in the library)
    return std::atoi(e) == static_cast<int>(dev::kDecodeFixedCheck) ? 1u : 0u;
}

#ifdef HUFF_STAMPS
// Timing builds only (tools/build_variant.sh -DHUFF_STAMPS): per-wave phase
// stamps of the index-free speculative pass (region 0), the skip decoder
// (region 1) and the indexed decoder (region 2), 10 words per wave
// (bitreader.hpp WaveStamps); huff_diag_stamps copies a region out.
constexpr size_t kStampRegionWords = 8u << 20;  // 64 MiB per region: >= 800 K waves
static uint64_t* g_stamps = nullptr;
uint64_t* stamp_region(int r) {
    if (!g_stamps && hipMalloc(&g_stamps, 3 * kStampRegionWords * 8) != hipSuccess) g_stamps = nullptr;
    if (!g_stamps) return nullptr;
    return g_stamps + r * kStampRegionWords;
}
#endif

// a checked k_decode_fixed launch: zero the mismatch record before, read it
// after (a host wait: test builds only)
Status run_checked_decode(huff_ctx* ctx, dev::DecodeArgs& a, const std::function<hipError_t()>& launch) {
#ifdef HUFF_STAMPS
    a.stamps = stamp_region(a.skip_packed ? 1 : 2);
#endif
    if (!a.check_mode) return hip_status(launch(), "decode");
    HUFF_TRY(ctx->d_err.ensure(32));
    a.err = static_cast<uint32_t*>(ctx->d_err.p);
    HIP_TRY(hipMemsetAsync(a.err, 0, 32, ctx->stream));
    HIP_TRY(launch());
    uint32_t e[8] = {};
    HIP_TRY(hipMemcpyAsync(e, a.err, 32, hipMemcpyDeviceToHost, ctx->stream));
    HUFF_TRY(ctx->sync());
    if (e[0] == 0) return Status::ok();
    const uint64_t want = (static_cast<uint64_t>(e[4]) << 32) | e[3], got = (static_cast<uint64_t>(e[6]) << 32) | e[5];
    return Status::err(HUFF_E_CORRUPT, "decode self-check: " + std::to_string(e[0]) + " lane(s) did not end at their "
                       "successor's restart point; first: task " + std::to_string(e[1]) + " lane " +
                       std::to_string(e[2]) + " ended at bit " + std::to_string(got) + ", expected " +
                       std::to_string(want));
}

// The decode tables are built once per tree, on the host, between pass 1 and
// the decode. Each used to walk the tree bit by bit for every one of its 2^K
// windows (~0.2 ms uniform, ~0.45 ms Zipf on this container's CPU), which at
// 128 MiB per rank outlasted the pack it hides behind; they are now filled
// from the tree's top K levels once (O(2^K + nodes)) and the walk table by a
// recurrence over window prefixes.

// the top K levels of the tree (K = sbits): entry i of `single` is the first
// code of the K-bit window i (MSB first) as decompress walks it
// (comp.rs:487-519): len | letter << 8, or kSsSlow when the window ends on an
// internal node (listed in `slow` with that node, ascending window order)
static void top_levels(const HuffTree& t, uint32_t K, uint16_t* single,
                       std::vector<std::pair<uint32_t, int32_t>>* slow) {
    const auto& nodes = t.nodes();
    const uint32_t n = 1u << K;
    if (t.root_is_leaf()) {  // every bit decodes the root letter (comp.rs:506-509)
        const uint16_t e = static_cast<uint16_t>(1u | (static_cast<uint32_t>(nodes[t.root()].letter) << 8));
        for (uint32_t i = 0; i < n; ++i) single[i] = e;
        return;
    }
    struct F {
        int32_t node;
        uint32_t depth, path;
    };
    std::vector<F> st{{t.root(), 0, 0}};
    while (!st.empty()) {
        const F f = st.back();
        st.pop_back();
        const HuffNode& nd = nodes[f.node];
        if (f.depth && nd.is_leaf) {
            const uint16_t e = static_cast<uint16_t>(f.depth | (static_cast<uint32_t>(nd.letter) << 8));
            const uint32_t lo = f.path << (K - f.depth), hi = (f.path + 1) << (K - f.depth);
            for (uint32_t i = lo; i < hi; ++i) single[i] = e;
        } else if (f.depth == K) {
            single[f.path] = static_cast<uint16_t>(dev::kSsSlow);
            if (slow) slow->push_back({f.path, f.node});
        } else {  // right first on the stack: windows come out in ascending order
            st.push_back({nd.right, f.depth + 1, (f.path << 1) | 1});
            st.push_back({nd.left, f.depth + 1, f.path << 1});
        }
    }
}

// entry i of the single-symbol table: the first code of the sbits-bit window i
static void build_single_table(const HuffTree& t, uint32_t sbits, DecTables& out,
                               std::vector<std::pair<uint32_t, int32_t>>* slow = nullptr) {
    const uint32_t n = 1u << sbits;
    out.sbits = sbits;
    out.soff = static_cast<uint32_t>(out.lut.size());
    out.lut.resize(out.lut.size() + (n + 1) / 2, 0);
    top_levels(t, sbits, reinterpret_cast<uint16_t*>(out.lut.data() + out.soff), slow);
}

// entry i of the walk table: every complete code of the sbits-bit window i
// (bits used, count, the first code's length), for walking a stream without
// its letters. Over the windows' suffixes: the m-bit string v holds its
// first code (length l <= m, from the single table at v << (K - m)) and then
// the complete codes of its last m - l bits, so (count, used) of every
// m-bit string follow from those of shorter ones, m = 1 .. K.
static void build_walk_table(const HuffTree& t, uint32_t sbits, DecTables& out) {
    (void)t;
    const uint32_t K = sbits, n = 1u << K;
    out.woff = static_cast<uint32_t>(out.lut.size());
    out.lut.resize(out.lut.size() + (n + 1) / 2, 0);
    const uint16_t* single = reinterpret_cast<const uint16_t*>(out.lut.data() + out.soff);
    uint16_t* w = reinterpret_cast<uint16_t*>(out.lut.data() + out.woff);
    // cu[(1 << m) + v] = count | used << 8 of the m-bit string v
    std::vector<uint16_t> cu(size_t(2) << K, 0);
    for (uint32_t m = 1; m <= K; ++m) {
        uint16_t* row = cu.data() + (size_t(1) << m);
        for (uint32_t v = 0; v < (1u << m); ++v) {
            const uint32_t e = single[v << (K - m)];
            const uint32_t l = e & 63u;
            if ((e & dev::kSsSlow) || l > m) continue;  // no complete code
            const uint32_t r = cu[(size_t(1) << (m - l)) + (v & ((1u << (m - l)) - 1))];
            row[v] = static_cast<uint16_t>(((r & 0xFFu) + 1) | (((r >> 8) + l) << 8));
            if (m == K)
                w[v] = static_cast<uint16_t>(l | (((r >> 8) + l) << 8) | (((r & 0xFFu) + 1) << 12));
        }
    }
    for (uint32_t v = 0; v < n; ++v)
        if ((cu[n + v] & 0xFFu) == 0) w[v] = static_cast<uint16_t>(dev::kSsSlow);
}

// The sync kernels' level-2 length table (DecTables::l2off): for every
// sbits-bit window whose first code is longer, the lengths of the codes below
// that node, indexed by exactly the E bits its deepest leaf needs; the slow
// entries of the single-symbol and walk tables get the descriptor index. Only
// the code lengths matter to the speculative pass and the marks, so a window
// that once took two dependent global reads (the 8-bit secondary tables) takes
// two LDS reads. Skipped past kL2MaxBytes (the LDS beside the stage) or for
// codes > 32 bits.
// Uniform form (DecTables::l2E) when it fits: every slow window gets 2^Emax
// lengths (Emax = the deepest leaf below any of them), so a slow step reads
// one length at index << Emax | next bits instead of a descriptor and then a
// length (two dependent LDS reads).
static void build_len_l2(const HuffTree& t, const std::vector<std::pair<uint32_t, int32_t>>& slow_nodes,
                         DecTables& out) {
    constexpr size_t kL2MaxBytes = 24 * 1024;
    constexpr uint32_t kMaxDesc = 1u << 15;
    const uint32_t K = out.sbits;
    if (t.root_is_leaf() || out.maxdepth <= K || out.maxdepth > 32) return;
    const auto& nodes = t.nodes();
    struct Slow {
        uint32_t window;
        int32_t node;
        uint32_t E;  // the deepest leaf below node, relative to it
    };
    std::vector<Slow> slow;
    uint32_t Emax = 0;
    size_t desc_bytes = 0;
    for (const auto& [i, x] : slow_nodes) {
        uint32_t E = 0;
        std::vector<std::pair<int32_t, uint32_t>> st{{x, 0}};
        while (!st.empty()) {
            auto [y, d] = st.back();
            st.pop_back();
            if (nodes[y].is_leaf) {
                E = std::max(E, d);
            } else {
                st.push_back({nodes[y].left, d + 1});
                st.push_back({nodes[y].right, d + 1});
            }
        }
        if (slow.size() >= kMaxDesc || K + E > 32) return;
        slow.push_back({i, x, E});
        Emax = std::max(Emax, E);
        desc_bytes += 4 + (size_t(1) << E);
    }
    if (slow.empty()) return;
    const bool uniform = (slow.size() << Emax) <= kL2MaxBytes;
    if (!uniform && desc_bytes > kL2MaxBytes) return;
    // the length of the code below `x` whose next E bits are j
    auto len_below = [&](int32_t x, uint32_t E, uint32_t j) {
        int32_t y = x;
        for (uint32_t p = 0; p < E; ++p) {
            y = ((j >> (E - 1 - p)) & 1u) ? nodes[y].right : nodes[y].left;
            if (nodes[y].is_leaf) return static_cast<uint8_t>(K + p + 1);
        }
        return static_cast<uint8_t>(K + E);
    };
    std::vector<uint8_t> b;
    if (uniform) {
        out.l2E = Emax;
        out.l2dense = slow.size() * 64 > (size_t(1) << K) && !std::getenv("HUFF_L2_SPARSE");  // (A/B: =1 branches)
        b.resize(slow.size() << Emax);
        for (size_t s = 0; s < slow.size(); ++s)
            for (uint32_t j = 0; j < (1u << Emax); ++j) b[(s << Emax) + j] = len_below(slow[s].node, Emax, j);
    } else {  // descriptors (byte offset << 5 | E), then each window's 2^E lengths
        out.l2E = 0;
        b.resize(slow.size() * 4);
        for (size_t s = 0; s < slow.size(); ++s) {
            const uint32_t d = static_cast<uint32_t>((b.size() << 5) | slow[s].E);
            std::memcpy(&b[s * 4], &d, 4);
            for (uint32_t j = 0; j < (1u << slow[s].E); ++j) b.push_back(len_below(slow[s].node, slow[s].E, j));
        }
    }
    out.l2off = static_cast<uint32_t>(out.lut.size());
    out.l2words = static_cast<uint32_t>((b.size() + 15) / 16 * 4);
    out.lut.resize(out.lut.size() + out.l2words, 0);
    std::memcpy(out.lut.data() + out.l2off, b.data(), b.size());
    std::vector<std::pair<uint32_t, uint32_t>> slow_ix;  // (window, index)
    for (size_t s = 0; s < slow.size(); ++s) slow_ix.push_back({slow[s].window, static_cast<uint32_t>(s)});
    uint16_t* s = reinterpret_cast<uint16_t*>(out.lut.data() + out.soff);
    uint16_t* w = reinterpret_cast<uint16_t*>(out.lut.data() + out.woff);
    for (auto [i, d] : slow_ix) {
        const uint16_t e = static_cast<uint16_t>(dev::kSsSlow | (d & 0x7Fu) | ((d >> 7) << 8));
        s[i] = e;
        w[i] = e;
    }
}

Status build_dec_tables(const HuffTree& t, DecTables& out) {
    const auto& nodes = t.nodes();
    out.lut.clear();
    out.l2off = out.l2words = out.l2E = 0;
    out.l2dense = false;
    if (t.root_is_leaf()) {  // every bit decodes the root letter (comp.rs:506-509)
        out.bits = 1;
        out.maxdepth = 1;
        const uint32_t e = (1u << 8) | nodes[t.root()].letter;
        out.lut = {e, e};
        build_single_table(t, 1, out);
        build_walk_table(t, 1, out);
        return Status::ok();
    }
    uint32_t mind = 0, maxd = 0;  // maxd > dev::kLongMaxLen: the deep kernels (deep.hip)
    t.depth_range(&mind, &maxd);
    out.maxdepth = maxd;
    out.all8 = (mind == 8 && maxd == 8);
    out.bits = std::min<uint32_t>(maxd, dev::kLutMaxBits - 1);  // 11 bits: 8 KiB of LDS
    if (out.bits < 1) out.bits = 1;
    out.lut.assign(1u << out.bits, 0);

    // fill the table rooted at internal node `x` (depth d0, tb index bits)
    struct Job {
        int32_t x;
        uint32_t d0, tb, base;
    };
    std::vector<Job> jobs{{t.root(), 0, out.bits, 0}};
    while (!jobs.empty()) {
        Job j = jobs.back();
        jobs.pop_back();
        struct F {
            int32_t node;
            uint32_t r;
            uint32_t path;
        };
        std::vector<F> st{{nodes[j.x].right, 1, 1}, {nodes[j.x].left, 1, 0}};
        while (!st.empty()) {
            F f = st.back();
            st.pop_back();
            const HuffNode& nd = nodes[f.node];
            if (nd.is_leaf) {
                const uint32_t e = ((j.d0 + f.r) << 8) | nd.letter;
                const uint32_t lo = f.path << (j.tb - f.r), hi = (f.path + 1) << (j.tb - f.r);
                for (uint32_t i = lo; i < hi; ++i) out.lut[j.base + i] = e;
            } else if (f.r == j.tb) {
                const uint32_t sub = static_cast<uint32_t>(out.lut.size());
                out.lut.resize(out.lut.size() + 256, 0);
                out.lut[j.base + f.path] = dev::kLutPtr | sub;
                jobs.push_back({f.node, j.d0 + j.tb, 8, sub});
            } else {
                st.push_back({nd.right, f.r + 1, (f.path << 1) | 1});
                st.push_back({nd.left, f.r + 1, f.path << 1});
            }
        }
    }
    std::vector<std::pair<uint32_t, int32_t>> slow;  // the single table's slow windows and their nodes
    build_single_table(t, std::min<uint32_t>(maxd, dev::kSsMaxBits), out, &slow);
    if (slow.empty()) {
        const uint16_t* st = reinterpret_cast<const uint16_t*>(out.lut.data() + out.soff);
        uint64_t sum = 0;
        for (uint32_t i = 0; i < (1u << out.sbits); ++i) sum += st[i] & 63u;
        out.kraft_bits = static_cast<double>(sum) / static_cast<double>(1u << out.sbits);
    }
    build_walk_table(t, out.sbits, out);
    build_len_l2(t, slow, out);
    return Status::ok();
}

}  // namespace huff

// ---------------------------------------------------------------------------
// buffers
// ---------------------------------------------------------------------------
huff::Status PinnedBuf::ensure(size_t bytes) {
    if (bytes <= cap) return wait();
    HUFF_TRY(wait());
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t c = std::max<size_t>(bytes, 4096);
    HIP_TRY(hipHostMalloc(&p, c, hipHostMallocDefault));
    cap = c;
    if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    return huff::Status::ok();
}

huff::Status PinnedBuf::wait() {
    if (!ev) return huff::Status::ok();
    // spin briefly (the waits here guard ~10 us copies on the critical path
    // between pass 1 and pass 2), then block
    for (int i = 0; i < 200000; ++i) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) return huff::Status::ok();
        if (q != hipErrorNotReady) HIP_TRY(q);
    }
    HIP_TRY(hipEventSynchronize(ev));
    return huff::Status::ok();
}

PinnedBuf::~PinnedBuf() {
    if (ev) {
        hipEventSynchronize(ev);
        hipEventDestroy(ev);
    }
    if (p) hipHostFree(p);
}

huff::Status DevBuf::ensure(size_t bytes) {
    if (bytes <= cap && p) return huff::Status::ok();
    release();
    size_t c = std::max<size_t>((bytes + 255) & ~size_t(255), 256);
    HIP_TRY(hipMalloc(&p, c));
    cap = c;
    return huff::Status::ok();
}

void DevBuf::release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
}

// ---------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------
huff::Status huff_ctx::activate() const {
    HIP_TRY(hipSetDevice(device));
    return huff::Status::ok();
}

huff::dev::LaunchEvents& huff::dev::launch_events() {
    static thread_local LaunchEvents e;
    return e;
}

huff::Status huff_ctx::timed(const char* name, const std::function<hipError_t()>& launch) {
    if (!timing) {
        HIP_TRY(launch());
        return huff::Status::ok();
    }
    hipEvent_t ev[2];
    for (auto& e : ev) {
        if (!free_events.empty()) {
            e = free_events.back();
            free_events.pop_back();
        } else {
            // HUFF_TIME_FENCE=none|device: events without the system-scope
            // fence on completion (A/B: step time within noise of the
            // default, profiles/r06/timing)
            static const unsigned flags = [] {
                const char* f = std::getenv("HUFF_TIME_FENCE");
                if (f && !std::strcmp(f, "none")) return unsigned(hipEventDisableSystemFence);
                if (f && !std::strcmp(f, "device")) return unsigned(hipEventReleaseToDevice);
                return 0u;
            }();
            HIP_TRY(hipEventCreateWithFlags(&e, flags));
        }
    }
    // the region's launches carry the pair themselves (kernels.hpp launch_k);
    // a region that launched nothing gets two markers, as does HUFF_TIME_MARKERS=1
    static const bool markers = [] {
        const char* m = std::getenv("HUFF_TIME_MARKERS");
        return m && *m == '1';
    }();
    auto& le = huff::dev::launch_events();
    if (markers) HIP_TRY(hipEventRecord(ev[0], stream));
    else le = {ev[0], ev[1]};
    const hipError_t err = launch();
    const bool none = le.start != nullptr;
    le = {};
    HIP_TRY(err);
    if (none && !markers) HIP_TRY(hipEventRecord(ev[0], stream));
    if (none || markers) HIP_TRY(hipEventRecord(ev[1], stream));
    pending.push_back({name, ev[0], ev[1]});
    return huff::Status::ok();
}

huff::Status huff_ctx::collect_timing() {
    if (pending.empty()) return huff::Status::ok();
    HIP_TRY(hipStreamSynchronize(stream));
    for (auto& p : pending) {
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, p.a, p.b));
        auto& k = kstats[p.name];
        k.first += ms;
        k.second += 1;
        free_events.push_back(p.a);
        free_events.push_back(p.b);
    }
    pending.clear();
    return huff::Status::ok();
}

huff::Status huff_ctx::sync() {
    HIP_TRY(hipStreamSynchronize(stream));
    return huff::Status::ok();
}

huff::Status huff_ctx::upload_dec_tables(const huff_tree* t, const huff::DecTables** dt, bool for_decode) {
    HUFF_TRY(t->dec_tables(dt));
    if (lut_tree_id == t->id) return huff::Status::ok();
    // no copy and no cross-stream wait in front of a byte-map decode (~5 us
    // of idle before it on the headline step)
    if (for_decode && (*dt)->all8 && !huff::fixed8_disabled()) return huff::Status::ok();
    const size_t bytes = (*dt)->lut.size() * 4;
    HUFF_TRY(pin_lut.ensure(bytes));  // waits until the previous upload has left it
    std::memcpy(pin_lut.p, (*dt)->lut.data(), bytes);
    HUFF_TRY(d_lut.ensure(bytes));
    // the copy runs on the side stream, beside what is already queued (the
    // pack of this job), once the last kernel that read d_lut is done; the
    // main stream waits for it before the next kernel
    HIP_TRY(hipStreamWaitEvent(copy_stream, lut_free, 0));
    HIP_TRY(hipMemcpyAsync(d_lut.p, pin_lut.p, bytes, hipMemcpyHostToDevice, copy_stream));
    HIP_TRY(hipEventRecord(pin_lut.ev, copy_stream));
    HIP_TRY(hipStreamWaitEvent(stream, pin_lut.ev, 0));
    lut_tree_id = t->id;
    return huff::Status::ok();
}

// ---------------------------------------------------------------------------
// encode job
// ---------------------------------------------------------------------------
huff::Status huff_enc::init(huff_ctx* c, const uint8_t* d, uint64_t nbytes) {
    if (reinterpret_cast<uintptr_t>(d) & 15)
        return huff::Status::err(HUFF_E_INVALID_ARG, "device input must be 16-byte aligned");
    if (nbytes >= (1ull << 48))  // pass 1 publishes 48-bit totals (hist.hip, k_hist_publish)
        return huff::Status::err(HUFF_E_INVALID_ARG, "one job holds fewer than 2^48 bytes");
    ctx = c;
    d_in = d;
    n = nbytes;
    nchunks = static_cast<uint32_t>((n + huff::dev::kChunk - 1) / huff::dev::kChunk);
    have_hist = packed = sums_valid = false;
    const size_t nc = std::max<uint32_t>(nchunks, 1);
    HUFF_TRY(chunk_hist.ensure(nc * 256 * 4));
    HUFF_TRY(gw.ensure(huff::dev::kHistCopies * 256 * 8 + 8));  // + k_rows_publish's ticket

    HUFF_TRY(chunk_bits.ensure(nc * 8));
    HUFF_TRY(chunk_start.ensure((nc + 1) * 8));
    HUFF_TRY(tsum.ensure((nc / 1024 + 2) * 8));
    HUFF_TRY(sub_bit.ensure(((n + huff::dev::kIdx - 1) / huff::dev::kIdx + 1) * 4));
    HUFF_TRY(mask.ensure(256));
    HUFF_TRY(pos.ensure(8));
    return huff::Status::ok();
}

// Host waits on a tagged pinned word (pass 1's weights, the index-free
// totals). hipStreamQuery on a stream whose work is still running queues a
// marker behind that work, which left ~6 us of idle in front of the next
// kernel (profiles/r06/pipeline). The liveness check (did the stream end
// without publishing? did a kernel fault?) therefore runs only once a wait
// has outlasted 2 ms, then once a millisecond, yielding the core between.
class SpinWait {
public:
    bool check_due() {
        if ((++spin_ & 255) != 0) return false;
        const auto now = std::chrono::steady_clock::now();
        if (now - t0_ < std::chrono::milliseconds(2)) return false;
        std::this_thread::yield();
        if (now - last_ < std::chrono::milliseconds(1)) return false;
        last_ = now;
        return true;
    }

private:
    std::chrono::steady_clock::time_point t0_ = std::chrono::steady_clock::now(), last_{};
    uint64_t spin_ = 0;
};

huff::Status huff_enc::launch_publish(uint64_t* tag) {
    HUFF_TRY(ctx->pin_w.ensure(256 * 8));
    if (!ctx->pin_w_dev) {
        std::memset(ctx->pin_w.p, 0, 256 * 8);
        HIP_TRY(hipHostGetDevicePointer(&ctx->pin_w_dev, ctx->pin_w.p, 0));
    }
    huff::dev::HistDone done;
    done.host = static_cast<unsigned long long*>(ctx->pin_w_dev);
    ctx->hist_seq = (ctx->hist_seq % 0xFFFF) + 1;  // 1..65535: never the zeroed buffer's tag
    done.tag = ctx->hist_seq;
    HUFF_TRY(ctx->timed("hist", [&] {
        return huff::dev::launch_hist(d_in, 0, n, nchunks, static_cast<uint32_t*>(chunk_hist.p),
                                      static_cast<unsigned long long*>(gw.p), ctx->stream, done);
    }));
    *tag = done.tag;
    return huff::Status::ok();
}

huff::Status huff_enc::wait_weights(uint64_t tag) {
    // every word carries the launch's tag once written (k_hist_publish)
    const uint64_t* hw = static_cast<const uint64_t*>(ctx->pin_w.p);
    hipStream_t s = ctx->stream;
    int b = 0;
    SpinWait sw;
    while (b < 256) {
        const uint64_t v = __atomic_load_n(&hw[b], __ATOMIC_ACQUIRE);
        if ((v >> 48) == tag) {
            w[b++] = v & ((1ull << 48) - 1);
            continue;
        }
        if (sw.check_due()) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess && (__atomic_load_n(&hw[b], __ATOMIC_ACQUIRE) >> 48) != tag)
                return huff::Status::err(HUFF_E_HIP, "pass 1 finished without publishing its weights");
            if (q != hipSuccess && q != hipErrorNotReady) HIP_TRY(q);
        }
    }
    return huff::Status::ok();
}

// the context's pinned weights word serves one pending pass 1 at a time
static huff::Status pending_guard(const huff_ctx* ctx, const huff_enc* e) {
    if (ctx->hist_pending && ctx->hist_pending != e)
        return huff::Status::err(HUFF_E_STATE, "another job's pass 1 is pending on this context (huff_enc_hist_launch): "
                                               "compress or hist that job first");
    return huff::Status::ok();
}

huff::Status huff_enc::hist_launch() {
    HUFF_TRY(ctx->activate());
    HUFF_TRY(pending_guard(ctx, this));
    if (nchunks == 0 || ctx->hist_pending == this) return huff::Status::ok();
    uint64_t tag = 0;
    HUFF_TRY(launch_publish(&tag));
    ctx->hist_pending = this;
    ctx->hist_pending_tag = tag;
    return huff::Status::ok();
}

huff::Status huff_enc::hist() {
    HUFF_TRY(ctx->activate());
    HUFF_TRY(pending_guard(ctx, this));
    if (nchunks == 0) {
        for (int b = 0; b < 256; ++b) w[b] = 0;
        have_hist = true;
        packed = false;
        return huff::Status::ok();
    }
    uint64_t tag = 0;
    if (ctx->hist_pending == this) {  // queued ahead: only the wait is left
        tag = ctx->hist_pending_tag;
        ctx->hist_pending = nullptr;
    } else {
        HUFF_TRY(launch_publish(&tag));
    }
    HUFF_TRY(wait_weights(tag));
    have_hist = true;
    packed = false;
    return huff::Status::ok();
}

huff::Status huff_enc::hist_known(const uint64_t counts[256]) {
    HUFF_TRY(ctx->activate());
    if (ctx->hist_pending == this) ctx->hist_pending = nullptr;  // its weights are not wanted now
    std::memcpy(w, counts, sizeof w);
    have_hist = true;
    packed = false;
    if (nchunks == 0) return huff::Status::ok();
    return ctx->timed("hist", [&] {
        return huff::dev::launch_hist(d_in, 0, n, nchunks, static_cast<uint32_t*>(chunk_hist.p),
                                      static_cast<unsigned long long*>(gw.p), ctx->stream);
    });
}

huff::Status huff_enc::hist_row(long long* d_row) {
    HUFF_TRY(ctx->activate());
    if (ctx->hist_pending == this) ctx->hist_pending = nullptr;
    hipStream_t s = ctx->stream;
    // the restart index (and the check build's sums) still describe the last
    // packed stream until the next pack rewrites them: a decode of that
    // stream may still be queued after this pass 1 (huff_mgpu_exchange_launch)
    have_hist = false;
    if (nchunks == 0) {
        HIP_TRY(hipMemsetAsync(d_row, 0, 258 * 8, s));
        return huff::Status::ok();
    }
    HUFF_TRY(ctx->timed("hist", [&] {
        hipError_t e = huff::dev::launch_hist(d_in, 0, n, nchunks, static_cast<uint32_t*>(chunk_hist.p),
                                              static_cast<unsigned long long*>(gw.p), s);
        if (e != hipSuccess) return e;
        return huff::dev::launch_hist_row(static_cast<const unsigned long long*>(gw.p), d_in, n, d_row, s);
    }));
    return huff::Status::ok();
}

huff::Status huff_enc::bits(const huff_tree* t, uint64_t* total) {
    if (!have_hist) return huff::Status::err(HUFF_E_STATE, "huff_enc_hist must run before bits/pack");
    const huff::EncTables& et = t->enc_tables();
    uint64_t b = 0;
    for (int i = 0; i < 256; ++i) {
        if (w[i] && et.len[i] == 0) {
            // compress_with_tree reports the FIRST missing letter in input order
            uint8_t m[256];
            for (int k = 0; k < 256; ++k) m[k] = (w[k] && et.len[k] == 0) ? 1 : 0;
            HUFF_TRY(ctx->activate());
            HIP_TRY(hipMemcpy(mask.p, m, 256, hipMemcpyHostToDevice));
            unsigned long long init = ~0ull;
            HIP_TRY(hipMemcpy(pos.p, &init, 8, hipMemcpyHostToDevice));
            HIP_TRY(huff::dev::launch_find_first(d_in, n, static_cast<const uint8_t*>(mask.p),
                                                 static_cast<unsigned long long*>(pos.p), ctx->stream));
            unsigned long long p = 0;
            HIP_TRY(hipMemcpyAsync(&p, pos.p, 8, hipMemcpyDeviceToHost, ctx->stream));
            HUFF_TRY(ctx->sync());
            uint8_t letter = 0;
            HIP_TRY(hipMemcpy(&letter, d_in + p, 1, hipMemcpyDeviceToHost));
            huff::Status st = huff::Status::err(HUFF_E_MISSING_LETTER, "letter not found in codes");
            st.missing_letter = letter;
            return st;
        }
        b += w[i] * et.len[i];
    }
    *total = b;
    return huff::Status::ok();
}

// the check build's letter checksums of the decoded job (checksum.hip): a
// wrong letter whose code has the right length keeps the stream in step, so
// only this sees it
huff::Status huff_enc::check_sums(const uint8_t* d_out) {
    if (!sums_valid || !huff::decode_check_mode()) return huff::Status::ok();
    HUFF_TRY(ctx->d_err.ensure(32));
    unsigned int* err = static_cast<unsigned int*>(ctx->d_err.p);
    const unsigned int init[2] = {0u, ~0u};
    HIP_TRY(hipMemcpyAsync(err, init, 8, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(huff::dev::launch_task_sums_check(d_out, n, static_cast<const uint64_t*>(task_sums.p), err, ctx->stream));
    unsigned int e[2] = {};
    HIP_TRY(hipMemcpyAsync(e, err, 8, hipMemcpyDeviceToHost, ctx->stream));
    HUFF_TRY(ctx->sync());
    if (e[0] == 0) return huff::Status::ok();
    return huff::Status::err(HUFF_E_CORRUPT, "decode self-check: letter checksums differ in " + std::to_string(e[0]) +
                                                 " task(s) of 4096 letters; first: task " + std::to_string(e[1]));
}

huff::PackStamps& huff::pack_stamps() {
    static thread_local PackStamps p;
    return p;
}

huff::Status huff_enc::pack(const huff_tree* t, uint64_t base, const uint8_t* prev_tail, size_t prev_tail_len,
                            uint8_t* d_out, size_t out_cap, uint64_t* total) {
    auto& ps = huff::pack_stamps();
    ps.bits = ps.launch = ps.launched = {};
    uint64_t tb = 0;
    HUFF_TRY(bits(t, &tb));
    ps.bits = std::chrono::steady_clock::now();
    compact_index = false;  // set by the general pack below when it writes the compact index
    const uint64_t need = ((base & 7) + tb + 7) / 8;
    if (total) *total = tb;
    if (need > out_cap) return huff::Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
    if (prev_tail_len > 8) return huff::Status::err(HUFF_E_INVALID_ARG, "prev_tail holds at most 8 bytes");
    HUFF_TRY(ctx->activate());
    hipStream_t s = ctx->stream;
    // the check build records the input's letter checksums for decode (checksum.hip)
    sums_valid = false;
    if (huff::decode_check_mode() && n) {
        HUFF_TRY(task_sums.ensure(((n + huff::dev::kTaskSym - 1) / huff::dev::kTaskSym) * 8));
        HIP_TRY(huff::dev::launch_task_sums(d_in, n, static_cast<uint64_t*>(task_sums.p), s));
        sums_valid = true;
    }
    const huff::EncTables& et = t->enc_tables();
    const bool long_codes = et.maxlen > huff::dev::kShortMaxLen;
    if ((base & 7) == 0 && et.maxlen == 8 && !huff::fixed8_disabled()) {
        bool all8 = true;
        for (int b = 0; b < 256; ++b) all8 &= (w[b] == 0 || et.len[b] == 8);
        if (all8) {  // every code 8 bits: byte substitution (bytemap.hip)
            huff::dev::BytemapArgs m{};
            m.src = d_in;
            m.dst = d_out;
            m.n = n;
            for (int b = 0; b < 256; ++b) m.map[b] = static_cast<uint8_t>(et.code[b]);
            m.nchunks = nchunks;
            m.base_bits = 0;
            ps.launch = std::chrono::steady_clock::now();
            HUFF_TRY(ctx->timed("pack", [&] { return huff::dev::launch_bytemap(m, s); }));
            ps.launched = std::chrono::steady_clock::now();
            packed = true;
            index_pending = true;  // arithmetic: written only if a consumer needs it
            packed_tree_id = t->id;
            remember_tree(t);
            bit_base = base;
            total_bits = tb;
            return huff::Status::ok();
        }
    }
    huff::dev::CodeLens lens;
    std::memcpy(lens.len, et.len, 256);
    HUFF_TRY(ctx->timed("chunk_bits", [&] {
        return huff::dev::launch_chunk_bits(static_cast<const uint32_t*>(chunk_hist.p), nchunks, lens,
                                            static_cast<uint64_t*>(chunk_bits.p), s);
    }));
    HUFF_TRY(ctx->timed("scan", [&] {
        return huff::dev::launch_scan(static_cast<const uint64_t*>(chunk_bits.p), nchunks, base & 7,
                                      static_cast<uint64_t*>(chunk_start.p), static_cast<uint64_t*>(tsum.p), s);
    }));
    if (et.maxlen > huff::dev::kLongMaxLen) {  // deep codes (deep.hip): ORed into a zeroed output
        const uint64_t nb = ((base & 7) + tb + 7) / 8;
        HIP_TRY(hipMemsetAsync(d_out, 0, nb, s));
        if ((base & 7) && prev_tail_len) {
            // the first byte's leading bits end the previous letters' codes
            // (what k_pack's lane 0 recomputes from prev_tail)
            uint32_t byte0 = 0;
            int64_t pos = static_cast<int64_t>(base & 7);
            for (size_t j = prev_tail_len; j-- > 0 && pos > 0;) {
                const uint8_t b = prev_tail[j];
                const int64_t L = et.len[b];
                if (L == 0) break;
                for (int64_t q = std::max<int64_t>(pos - L, 0); q < pos; ++q) {
                    const int64_t k = q - (pos - L);  // code bit index
                    if ((et.deep[b * huff::dev::kDeepWords + k / 32] >> (31 - k % 32)) & 1u) byte0 |= 0x80u >> q;
                }
                pos -= L;
            }
            HIP_TRY(hipMemsetAsync(d_out, static_cast<int>(byte0), 1, s));
        }
        HUFF_TRY(deep_words.ensure(256 * huff::dev::kDeepWords * 4));
        HIP_TRY(hipMemcpyAsync(deep_words.p, et.deep.data(), 256 * huff::dev::kDeepWords * 4, hipMemcpyHostToDevice, s));
        huff::dev::DeepPackArgs d{};
        d.len = lens;
        d.words = static_cast<const uint32_t*>(deep_words.p);
        d.in = d_in;
        d.n = n;
        d.chunk_start = static_cast<const uint64_t*>(chunk_start.p);
        d.nchunks = nchunks;
        d.out = d_out;
        d.sub_bit = static_cast<uint32_t*>(sub_bit.p);
        HUFF_TRY(ctx->timed("pack", [&] { return huff::dev::launch_pack_deep(d, s); }));
        packed = true;
        index_pending = false;
        packed_tree_id = t->id;
        remember_tree(t);
        bit_base = base;
        total_bits = tb;
        return huff::Status::ok();
    }
    huff::dev::PackArgs a{};
    if (long_codes)
        for (int b = 0; b < 256; ++b) a.table.l[b] = (et.code[b] << 6) | et.len[b];
    else
        for (int b = 0; b < 256; ++b)  // left-aligned (pack.hip Entry<false>)
            a.table.s[b] = et.len[b] ? static_cast<uint32_t>(et.code[b] << (32 - et.len[b])) | et.len[b] : 0u;
    if (prev_tail_len) std::memcpy(a.prev_tail + 8 - prev_tail_len, prev_tail, prev_tail_len);
    a.in = d_in;
    a.n = n;
    a.chunk_start = static_cast<const uint64_t*>(chunk_start.p);
    a.nchunks = nchunks;
    a.out = d_out;
    a.sub_bit = static_cast<uint32_t*>(sub_bit.p);
    // codes <= 16 bits: the compact restart index (4,096 codes fit a u16 offset)
    const bool compact = !long_codes && et.maxlen <= 16;
    if (compact) {
        HUFF_TRY(sub16.ensure(((n + huff::dev::kIdx - 1) / huff::dev::kIdx + 1) * 2));
        HUFF_TRY(task_base.ensure(((n + huff::dev::kTaskSym - 1) / huff::dev::kTaskSym + 1) * 8));
        a.sub16 = static_cast<uint16_t*>(sub16.p);
        a.task_base = static_cast<uint64_t*>(task_base.p);
        a.sub_bit = nullptr;
    }
    a.prev_tail_len = static_cast<uint32_t>(prev_tail_len);
    // one wave round: <= round bytes * maxlen bits + a < 128-bit carry (+ the
    // 128-bit window past the last unit, which the OR emit may touch with zero)
    a.stage_words = (huff::dev::pack_round_bytes() / 32 * std::max<uint32_t>(et.maxlen, 1) + 12 + 3) & ~3u;
    a.max_len = et.maxlen;
    const size_t lds = huff::dev::pack_lds_bytes(long_codes, et.maxlen, a.stage_words);
    const uint32_t per_cu = huff::dev::pack_groups_per_cu(long_codes, et.maxlen, lds);
    const uint32_t wpg = huff::dev::pack_waves_per_group(long_codes);
    a.grid = std::max<uint32_t>(1, std::min<uint32_t>((nchunks + wpg - 1) / wpg, ctx->cu_count * per_cu));
    HUFF_TRY(ctx->timed("pack", [&] { return huff::dev::launch_pack(long_codes, a, s); }));
    packed = true;
    index_pending = false;
    compact_index = compact;
    packed_tree_id = t->id;
    remember_tree(t);
    bit_base = base;
    total_bits = tb;
    return huff::Status::ok();
}

huff::Status huff_enc::ensure_index() {
    if (!index_pending) return huff::Status::ok();
    HUFF_TRY(ctx->activate());
    HIP_TRY(huff::dev::launch_arith_index(n, nchunks, bit_base & 7, static_cast<uint64_t*>(chunk_start.p),
                                          static_cast<uint32_t*>(sub_bit.p), ctx->stream));
    index_pending = false;
    compact_index = false;
    return huff::Status::ok();
}

huff::Status huff_enc::expand_index() {
    if (!compact_index) return huff::Status::ok();
    HUFF_TRY(ctx->activate());
    HIP_TRY(huff::dev::launch_index_expand(n, static_cast<const uint64_t*>(task_base.p),
                                           static_cast<const uint16_t*>(sub16.p),
                                           static_cast<const uint64_t*>(chunk_start.p),
                                           static_cast<uint32_t*>(sub_bit.p), ctx->stream));
    compact_index = false;
    return huff::Status::ok();
}

huff::Status huff_enc::decode(const huff_tree* t, const uint8_t* d_comp, uint64_t comp_bytes, uint8_t* d_out) {
    if (!packed) return huff::Status::err(HUFF_E_STATE, "no restart index: pack (or upload an index) first");
    if (!codes_match(t))
        return huff::Status::err(HUFF_E_STATE, "decode tree differs from the tree the stream was packed (or its index "
                                               "uploaded) with");
    if (reinterpret_cast<uintptr_t>(d_comp) & 3)
        return huff::Status::err(HUFF_E_INVALID_ARG, "compressed stream must be 4-byte aligned");
    HUFF_TRY(ctx->activate());
    const huff::DecTables* dt = nullptr;
    HUFF_TRY(t->dec_tables(&dt));
    if (dt->all8 && (bit_base & 7) == 0 && !huff::fixed8_disabled()) {  // inverse byte substitution
        huff::dev::BytemapArgs m{};
        m.src = d_comp;
        m.dst = d_out;
        m.n = n;
        for (int b = 0; b < 256; ++b) m.map[b] = static_cast<uint8_t>(dt->lut[b]);  // entries (8 << 8) | letter
        HUFF_TRY(ctx->timed("decode", [&] { return huff::dev::launch_bytemap(m, ctx->stream); }));
        return check_sums(d_out);
    }
    HUFF_TRY(ctx->upload_dec_tables(t, &dt));
    HUFF_TRY(ensure_index());
    huff::dev::DecodeArgs a{};
    if (dt->maxdepth > huff::dev::kLongMaxLen) {  // deep codes (deep.hip)
        a.comp = d_comp;
        a.comp_bytes = comp_bytes;
        a.lut = static_cast<const uint32_t*>(ctx->d_lut.p);
        a.lut_bits = dt->bits;
        a.chunk_start = static_cast<const uint64_t*>(chunk_start.p);
        a.sub_bit = static_cast<const uint32_t*>(sub_bit.p);
        a.nchunks = nchunks;
        a.n = n;
        a.out = d_out;
        HUFF_TRY(ctx->timed("decode", [&] { return huff::dev::launch_decode_deep(a, ctx->stream); }));
        HIP_TRY(hipEventRecord(ctx->lut_free, ctx->stream));
        return huff::Status::ok();
    }
    a.comp = d_comp;
    a.comp_bytes = comp_bytes;
    a.lut = static_cast<const uint32_t*>(ctx->d_lut.p);
    a.lut_bits = dt->bits;
    a.lut_words = static_cast<uint32_t>(dt->lut.size());
    a.chunk_start = static_cast<const uint64_t*>(chunk_start.p);
    a.sub_bit = static_cast<const uint32_t*>(sub_bit.p);
    a.nchunks = nchunks;
    a.max_len = dt->maxdepth;
    // codes <= 32 bits: the fixed-count decoder (decode_wave.hip,
    // k_decode_fixed; the round-1 ring, multi-symbol and single-symbol
    // decoders were 1.2-1.9x slower and are retired); HUFF_DEC_VARIANT=11
    // runs its self-checking build. Longer codes: k_decode<LONG> (decode.hip).
    a.check_mode = huff::decode_check_mode();
    // the task decoder stores 16-B pieces: a misaligned output (e.g. a tensor
    // view at an odd offset) is decoded into an aligned buffer of the context
    // and copied on the stream
    uint8_t* dst = d_out;
    const bool fixed = dt->maxdepth <= 32;
    if (compact_index) {  // the task decoder reads it as is; k_decode<LONG> gets sub_bit
        if (fixed) {
            a.sub16 = static_cast<const uint16_t*>(sub16.p);
            a.task_base = static_cast<const uint64_t*>(task_base.p);
        } else {
            HUFF_TRY(expand_index());
        }
    }
    const bool bounce = fixed && (reinterpret_cast<uintptr_t>(d_out) & 15);
    if (bounce) {
        HUFF_TRY(ctx->d_align.ensure(n + 64));
        dst = static_cast<uint8_t*>(ctx->d_align.p);
    }
    a.cu_count = static_cast<uint32_t>(ctx->cu_count);
    a.pad_stage = huff::dev::fixed_decode_pad(total_bits, n);
    a.small_stage = huff::small_stage_enabled() && huff::dev::fixed_decode_small(total_bits, n);
    a.dma_stage = huff::dma_decode_enabled();
    a.stab = reinterpret_cast<const uint16_t*>(static_cast<const uint32_t*>(ctx->d_lut.p) + dt->soff);
    a.stab_bits = dt->sbits;
    a.n = n;
    a.out = dst;
#ifdef HUFF_STAMPS
    a.stamps = huff::stamp_region(2);
#endif
    if (a.check_mode) {
        HUFF_TRY(huff::run_checked_decode(ctx, a, [&] { return huff::dev::launch_decode(a, ctx->stream); }));
        HUFF_TRY(check_sums(dst));
    } else {
        HUFF_TRY(ctx->timed("decode", [&] { return huff::dev::launch_decode(a, ctx->stream); }));
    }
    HIP_TRY(hipEventRecord(ctx->lut_free, ctx->stream));
    if (bounce && n) HIP_TRY(hipMemcpyAsync(d_out, dst, n, hipMemcpyDeviceToDevice, ctx->stream));
    return huff::Status::ok();
}

huff::Status huff_enc::download_index(huff_index_host& idx) {
    HUFF_TRY(ensure_index());
    HUFF_TRY(expand_index());  // the host index (CompressData) keeps chunk_start + sub_bit
    idx.n = n;
    idx.chunk_start.resize(nchunks + 1);
    idx.sub_bit.resize((n + huff::dev::kIdx - 1) / huff::dev::kIdx);
    HUFF_TRY(ctx->activate());
    HIP_TRY(hipMemcpyAsync(idx.chunk_start.data(), chunk_start.p, idx.chunk_start.size() * 8, hipMemcpyDeviceToHost,
                           ctx->stream));
    if (!idx.sub_bit.empty())
        HIP_TRY(hipMemcpyAsync(idx.sub_bit.data(), sub_bit.p, idx.sub_bit.size() * 4, hipMemcpyDeviceToHost,
                               ctx->stream));
    return ctx->sync();
}

huff::Status huff_enc::upload_index(const huff_index_host& idx) {
    if (idx.n != n || idx.chunk_start.size() != nchunks + 1u)
        return huff::Status::err(HUFF_E_INVALID_ARG, "restart index does not match the job");
    sums_valid = false;  // no encode of this job's letters behind the index
    HUFF_TRY(ctx->activate());
    HIP_TRY(hipMemcpyAsync(chunk_start.p, idx.chunk_start.data(), idx.chunk_start.size() * 8, hipMemcpyHostToDevice,
                           ctx->stream));
    if (!idx.sub_bit.empty())
        HIP_TRY(hipMemcpyAsync(sub_bit.p, idx.sub_bit.data(), idx.sub_bit.size() * 4, hipMemcpyHostToDevice,
                               ctx->stream));
    HUFF_TRY(ctx->sync());
    packed = true;
    packed_any_tree = true;  // the caller vouches for the tree (huff_enc_upload_index)
    index_pending = false;
    compact_index = false;
    return huff::Status::ok();
}

void huff_enc::remember_tree(const huff_tree* t) {
    const huff::EncTables& et = t->enc_tables();
    std::memcpy(packed_len, et.len, sizeof packed_len);
    std::memcpy(packed_code, et.code, sizeof packed_code);
    packed_deep = et.deep;
    packed_any_tree = false;
}

bool huff_enc::codes_match(const huff_tree* t) const {
    if (packed_any_tree) return true;
    const huff::EncTables& et = t->enc_tables();
    return std::memcmp(packed_len, et.len, sizeof packed_len) == 0 &&
           std::memcmp(packed_code, et.code, sizeof packed_code) == 0 && packed_deep == et.deep;
}

// ---------------------------------------------------------------------------
// host-pointer pipelines
// ---------------------------------------------------------------------------
namespace huff {

static Status stage_input(huff_ctx* ctx, const uint8_t* bytes, size_t n) {
    HUFF_TRY(ctx->activate());
    HUFF_TRY(ctx->d_in.ensure(n + 16));
    if (n) HIP_TRY(hipMemcpyAsync(ctx->d_in.p, bytes, n, hipMemcpyHostToDevice, ctx->stream));
    return Status::ok();
}

Status weights_from_host(huff_ctx* ctx, const uint8_t* bytes, size_t n, ByteWeights& out) {
    out = ByteWeights{};
    if (n == 0) return Status::ok();
    HUFF_TRY(stage_input(ctx, bytes, n));
    huff_enc e;
    HUFF_TRY(e.init(ctx, static_cast<const uint8_t*>(ctx->d_in.p), n));
    HUFF_TRY(e.hist());
    out = ByteWeights::from_counts(e.w);
    return Status::ok();
}

Status weights_threaded_from_host(huff_ctx* ctx, const uint8_t* bytes, size_t n, size_t thread_num,
                                  ByteWeights& out) {
    // weights.rs:293-319: per-ration histograms (here: one hist256 launch per
    // ration over the staged buffer), then `w = W_last; w += W_0 .. W_{T-2}`.
    if (thread_num == 0) return Status::err(HUFF_E_INVALID_ARG, "thread_num must be > 0");
    auto rations = ration_bounds(n, thread_num);
    HUFF_TRY(stage_input(ctx, bytes, n));
    const size_t R = rations.size();
    DevBuf gws;
    HUFF_TRY(gws.ensure(R * dev::kHistCopies * 256 * 8));
    HIP_TRY(hipMemsetAsync(gws.p, 0, R * dev::kHistCopies * 256 * 8, ctx->stream));
    const uint8_t* d = static_cast<const uint8_t*>(ctx->d_in.p);
    for (size_t r = 0; r < R; ++r) {
        const size_t lo = rations[r].first, hi = rations[r].second;
        if (hi == lo) continue;
        const size_t abase = lo & ~size_t(15);
        const uint64_t llo = lo - abase, lhi = hi - abase;
        const uint32_t nch = static_cast<uint32_t>((lhi + dev::kChunk - 1) / dev::kChunk);
        HIP_TRY(dev::launch_hist(d + abase, llo, lhi, nch, nullptr,
                                 static_cast<unsigned long long*>(gws.p) + r * dev::kHistCopies * 256, ctx->stream));
    }
    std::vector<uint64_t> h(R * dev::kHistCopies * 256);
    HIP_TRY(hipMemcpyAsync(h.data(), gws.p, h.size() * 8, hipMemcpyDeviceToHost, ctx->stream));
    HUFF_TRY(ctx->sync());
    std::vector<ByteWeights> parts(R);
    for (size_t r = 0; r < R; ++r) {
        uint64_t c[256];
        for (int b = 0; b < 256; ++b) {
            uint64_t s = 0;
            for (uint32_t k = 0; k < dev::kHistCopies; ++k) s += h[(r * dev::kHistCopies + k) * 256 + b];
            c[b] = s;
        }
        parts[r] = ByteWeights::from_counts(c);
    }
    out = parts[R - 1];
    for (size_t r = 0; r + 1 < R; ++r) out.add(parts[r]);
    return Status::ok();
}

Status compress_host(huff_ctx* ctx, const uint8_t* bytes, size_t n, const huff_tree* t, huff_compress_data** out) {
    *out = nullptr;
    if (n == 0) return Status::err(HUFF_E_EMPTY_COMP, "provided comp_bytes are empty");
    HUFF_TRY(stage_input(ctx, bytes, n));
    huff_enc e;
    HUFF_TRY(e.init(ctx, static_cast<const uint8_t*>(ctx->d_in.p), n));
    HUFF_TRY(e.hist());
    std::unique_ptr<huff_tree> own;
    if (!t) {  // compress_bytes: the tree comes from this very histogram
        own = std::make_unique<huff_tree>();
        HUFF_TRY(HuffTree::from_weights(ByteWeights::from_counts(e.w), own->t));
        t = own.get();
    }
    uint64_t tb = 0;
    HUFF_TRY(e.bits(t, &tb));
    const size_t nbytes = static_cast<size_t>((tb + 7) / 8);
    HUFF_TRY(ctx->d_out.ensure(nbytes + 16));
    HUFF_TRY(e.pack(t, 0, nullptr, 0, static_cast<uint8_t*>(ctx->d_out.p), nbytes, &tb));
    auto cd = std::make_unique<huff_compress_data>();
    cd->comp.resize(nbytes);
    HIP_TRY(hipMemcpyAsync(cd->comp.data(), ctx->d_out.p, nbytes, hipMemcpyDeviceToHost, ctx->stream));
    cd->padding = calc_padding_bits(tb);  // comp.rs:446
    cd->index = std::make_unique<huff_index_host>();
    HUFF_TRY(e.download_index(*cd->index));
    if (own) {
        cd->tree = own.release();
    } else {
        cd->tree = new huff_tree();
        cd->tree->t = t->t;
    }
    *out = cd.release();
    return Status::ok();
}

Status decompress_host(huff_ctx* ctx, const huff_compress_data* cd, uint8_t* out, size_t cap, size_t* out_len) {
    if (!cd->index) {
        // comp.rs:513-516: all bytes but the last give 8 bits, the last 8 - padding
        const uint64_t valid = static_cast<uint64_t>(cd->comp.size()) * 8 - cd->padding;
        std::vector<uint8_t> sym;
        HUFF_TRY(decode_indexless_host(ctx, cd->comp.data(), cd->comp.size(), valid, cd->tree, sym));
        *out_len = sym.size();
        if (cap < sym.size()) return Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
        if (!sym.empty()) std::memcpy(out, sym.data(), sym.size());
        return Status::ok();
    }
    const uint64_t n = cd->index->n;
    *out_len = n;
    if (cap < n) return Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
    if (n == 0) return Status::ok();
    HUFF_TRY(ctx->activate());
    HUFF_TRY(ctx->d_in.ensure(cd->comp.size() + 16));
    HIP_TRY(hipMemcpyAsync(ctx->d_in.p, cd->comp.data(), cd->comp.size(), hipMemcpyHostToDevice, ctx->stream));
    HUFF_TRY(ctx->d_out.ensure(n + 16));
    huff_enc e;
    // the job's input pointer is unused by decode; give it the output staging (aligned)
    HUFF_TRY(e.init(ctx, static_cast<const uint8_t*>(ctx->d_out.p), n));
    HUFF_TRY(e.upload_index(*cd->index));
    HUFF_TRY(e.decode(cd->tree, static_cast<const uint8_t*>(ctx->d_in.p), cd->comp.size(),
                      static_cast<uint8_t*>(ctx->d_out.p)));
    HIP_TRY(hipMemcpyAsync(out, ctx->d_out.p, n, hipMemcpyDeviceToHost, ctx->stream));
    return ctx->sync();
}

Status parse_block_size(const char* s, size_t* out) {
    // huff/src/cli.rs:79-114: digits, then an optional unit (case-insensitive)
    if (!s) return Status::err(HUFF_E_INVALID_ARG, "Invalid block size");
    std::string lower;
    for (const char* p = s; *p; ++p) lower.push_back(static_cast<char>(std::tolower(static_cast<unsigned char>(*p))));
    size_t i = 0;
    std::string num;
    while (i < lower.size() && std::isdigit(static_cast<unsigned char>(lower[i]))) num.push_back(lower[i++]);
    std::string mult = lower.substr(i);
    if (num.empty()) return Status::err(HUFF_E_INVALID_ARG, "Invalid block size");
    unsigned long long v = 0;
    for (char ch : num) {  // usize::parse: overflow is an error
        const unsigned d = static_cast<unsigned>(ch - '0');
        if (v > (~0ull - d) / 10) return Status::err(HUFF_E_INVALID_ARG, "Invalid block size");
        v = v * 10 + d;
    }
    if (v == 0) return Status::err(HUFF_E_INVALID_ARG, "Invalid block size");
    unsigned long long m;
    if (mult.empty()) m = 1;
    else if (mult == "k") m = 1000ull;
    else if (mult == "m") m = 1000000ull;
    else if (mult == "g") m = 1000000000ull;
    else if (mult == "ki") m = 1024ull;
    else if (mult == "mi") m = 1048576ull;
    else if (mult == "gi") m = 1073741824ull;
    else return Status::err(HUFF_E_INVALID_ARG, "Invalid block size");
    *out = static_cast<size_t>(v * m);
    return Status::ok();
}

}  // namespace huff

// ---------------------------------------------------------------------------
// index-free decode
// ---------------------------------------------------------------------------

huff::IndexlessSync& huff_ctx::indexless_ws() {
    if (!idx_ws) idx_ws = std::make_shared<huff::IndexlessSync>();
    return *idx_ws;
}

namespace huff {

Status indexless_sync(huff_ctx* ctx, const uint8_t* d_comp, uint64_t comp_bytes, uint64_t valid_bits,
                      const huff_tree* t, IndexlessSync& st, bool need_off,
                      const std::function<Status()>& before_wait) {
    const DecTables* dt = st.dt;
    // segment length: a multiple of the gcd of all code lengths
    uint32_t g = 0, lo_, hi_;
    t->t.depth_range(&lo_, &hi_, &g);
    if (g == 0) g = 1;
    // codes <= 32 bits take the LDS-staged kernels, longer codes 2048-bit segments
    // (~992 bits: with the one 8 KiB walk table a workgroup's LDS stays under
    // 40 KiB, 4 workgroups per CU; 1024-bit segments measured ~1.5 % slower)
#ifndef HUFF_SEG_TARGET
#define HUFF_SEG_TARGET 992
#endif
    const uint64_t seg_target = dt->maxdepth <= 32 ? HUFF_SEG_TARGET : 2048;
    uint64_t S = static_cast<uint64_t>(g) * ((seg_target + g - 1) / g);
    // the LDS-staged kernels read lane i's bits from dword ~S/32 * i: with an
    // even dword stride every lane starts on the same few banks (1024 bits: all
    // 32 lanes of a half-wave on one bank); prefer an odd stride (S = 32 mod 64)
    for (uint64_t k = (seg_target + g - 1) / g, tries = 0; tries < 128; ++k, ++tries)
        if ((static_cast<uint64_t>(g) * k) % 64 == 32) {
            S = static_cast<uint64_t>(g) * k;
            break;
        }
    // the staged kernels' sample words hold 10-bit offsets (indexless.hip)
    if (dt->maxdepth <= 32 && S >= 1024) S = static_cast<uint64_t>(g) * (1023 / g);
    const uint64_t nseg = (valid_bits + S - 1) / S;
    if (nseg > 0xFFFFFFFFull) return Status::err(HUFF_E_INVALID_ARG, "stream too long for one decode");
    HUFF_TRY(st.s.ensure(nseg * 8));
    HUFF_TRY(st.x0.ensure(nseg * 8));
    HUFF_TRY(st.c.ensure(nseg * 8));
    HUFF_TRY(st.off.ensure((nseg + 1) * 8));
    HUFF_TRY(st.tm.ensure(nseg * 4));
    HUFF_TRY(st.dl.ensure(nseg * 4));
    HUFF_TRY(st.flag.ensure(32));  // kFixRounds + 4 words, zeroed by one aligned fill
    const uint64_t nwg = (nseg + 255) / 256;  // workgroups of the staged speculative pass
    HUFF_TRY(st.wtot.ensure(nwg * 8));
    HUFF_TRY(st.woff.ensure((nwg + 1) * 8));
    dev::IndexlessArgs& a = st.a;
    a = dev::IndexlessArgs{};
    a.comp = d_comp;
    a.comp_bytes = comp_bytes;
    a.valid_bits = valid_bits;
    a.seg_bits = S;
    // in phase with the segment starts; longer for codes past the walk table
    a.lead_bits = (dt->maxdepth > dt->sbits ? dev::kLeadBitsLong : dev::kLeadBits) / g * g;
    a.nseg = nseg;
    a.lut = static_cast<const uint32_t*>(ctx->d_lut.p);
    a.lut_bits = dt->bits;
    a.s = static_cast<uint64_t*>(st.s.p);
    a.x = static_cast<uint64_t*>(st.x0.p);
    a.c = static_cast<uint64_t*>(st.c.p);
    a.max_len = dt->maxdepth;
    a.stab = reinterpret_cast<const uint16_t*>(static_cast<const uint32_t*>(ctx->d_lut.p) + dt->soff);
    a.stab_bits = dt->sbits;
    a.wtab = reinterpret_cast<const uint16_t*>(static_cast<const uint32_t*>(ctx->d_lut.p) + dt->woff);
    if (dt->l2words && !std::getenv("HUFF_NO_L2")) {  // HUFF_NO_L2=1: the global secondary tables (A/B)
        a.l2 = static_cast<const uint32_t*>(ctx->d_lut.p) + dt->l2off;
        a.l2_words = dt->l2words;
        a.l2_e = dt->l2E;
        a.l2_dense = dt->l2dense ? 1u : 0u;
    }
    a.tm = static_cast<uint32_t*>(st.tm.p);
    a.dl = static_cast<int32_t*>(st.dl.p);
    a.flags = static_cast<unsigned int*>(st.flag.p);
#ifdef HUFF_STAMPS
    a.stamps = stamp_region(0);
#endif
    hipStream_t strm = ctx->stream;
    if (dev::indexless_staged(a)) {  // speculative samples for the marking pass
        a.nsamp = std::min<uint32_t>(dev::kSampMax, static_cast<uint32_t>((S - 1) / dev::kSampBits));
        HUFF_TRY(st.samp.ensure(nseg * ((dev::kSampMax + 1) & ~1u) * 2 + 16));  // u16 slots, whole dwords per segment
        a.samp = static_cast<uint16_t*>(st.samp.p);
        HUFF_TRY(st.fixlist.ensure(nseg * 4 + 4));
        a.fixlist = static_cast<uint32_t*>(st.fixlist.p);
        HUFF_TRY(st.chain.ensure(nseg * 8 + 8));
        a.chain = static_cast<uint32_t*>(st.chain.p);
        HUFF_TRY(st.rec.ensure(nseg * 8));
        a.rec = static_cast<uint64_t*>(st.rec.p);
        a.wtot = static_cast<unsigned long long*>(st.wtot.p);
    } else {  // k_spec leaves the merge record to the fix-up rounds
        HIP_TRY(hipMemsetAsync(st.tm.p, 0, nseg * 4, strm));
        HIP_TRY(hipMemsetAsync(st.dl.p, 0, nseg * 4, strm));
    }
    static_assert((dev::kFixRounds + 4) * 4 <= 32, "the flags fit the zeroed 32 bytes");
    HIP_TRY(hipMemsetAsync(st.flag.p, 0, 32, strm));
    HIP_TRY(dev::launch_indexless_spec(a, strm));
    // fix-up rounds and the sequential fallback decide on the device whether
    // they have work (no host wait between rounds)
    HIP_TRY(dev::launch_indexless_settle_all(a, strm));
    HUFF_TRY(st.tsum.ensure((nseg / 1024 + 2) * 8));
    st.total = 0;
    // the staged pass keeps per-workgroup counts: only they are scanned
    // (k_mark_lite scans inside a workgroup), unless a consumer needs every
    // segment's offset (the walked marks, k_emit)
    st.block_off = a.wtot && !need_off;
    // the total goes from the scan's last kernel straight to pinned host
    // memory, tagged; the host polls it (a copy and a stream
    // synchronisation here cost ~40 us between the sync and the decode)
    HUFF_TRY(ctx->pin_total.ensure(8));
    if (!ctx->pin_total_dev) {
        std::memset(ctx->pin_total.p, 0, 8);
        HIP_TRY(hipHostGetDevicePointer(&ctx->pin_total_dev, ctx->pin_total.p, 0));
    }
    dev::HistDone done;
    done.host = static_cast<unsigned long long*>(ctx->pin_total_dev);
    ctx->total_seq = (ctx->total_seq % 0xFFFF) + 1;  // 1..65535: never the zeroed word's tag
    done.tag = ctx->total_seq;
    if (st.block_off) {
        HIP_TRY(dev::launch_scan(static_cast<const uint64_t*>(st.wtot.p), static_cast<uint32_t>(nwg), 0,
                                 static_cast<uint64_t*>(st.woff.p), static_cast<uint64_t*>(st.tsum.p), strm, done));
    } else {
        if (a.rec) HIP_TRY(dev::launch_indexless_counts(a, strm));  // the staged pass packs its counts
        HIP_TRY(dev::launch_scan(static_cast<const uint64_t*>(st.c.p), static_cast<uint32_t>(nseg), 0,
                                 static_cast<uint64_t*>(st.off.p), static_cast<uint64_t*>(st.tsum.p), strm, done));
    }
    if (before_wait) HUFF_TRY(before_wait());
    const uint64_t* hw = static_cast<const uint64_t*>(ctx->pin_total.p);
    SpinWait sw;
    for (;;) {
        const uint64_t v = __atomic_load_n(hw, __ATOMIC_ACQUIRE);
        if ((v >> 48) == done.tag) {
            // (a fault in the kernels before the scan stops the stream before
            // the scan publishes: the wait's liveness check reports it)
            st.total = v & ((1ull << 48) - 1);
            if (std::getenv("HUFF_FIX_STATS")) {  // diagnostics: how much the fix-up did (a synchronising copy)
                unsigned int f[8];
                HIP_TRY(hipMemcpyAsync(f, st.flag.p, sizeof f, hipMemcpyDeviceToHost, strm));
                HIP_TRY(hipStreamSynchronize(strm));
                std::fprintf(stderr, "huff fix-up: segments %llu, listed by the speculative pass %u, chain fixes %u\n",
                             static_cast<unsigned long long>(nseg), f[dev::kFixRounds], f[dev::kFixRounds + 3]);
            }
            return Status::ok();
        }
        if (sw.check_due()) {
            const hipError_t q = hipStreamQuery(strm);
            if (q == hipSuccess && (__atomic_load_n(hw, __ATOMIC_ACQUIRE) >> 48) != done.tag)
                return Status::err(HUFF_E_HIP, "the index-free scan finished without publishing its total");
            if (q != hipSuccess && q != hipErrorNotReady) HIP_TRY(q);
        }
    }
}

Status indexless_mark(huff_ctx* ctx, IndexlessSync& st, DevBuf& sub_abs, uint32_t shift) {
    HUFF_TRY(sub_abs.ensure(((st.total + (1ull << shift) - 1) >> shift) * 8 + 8));
    HIP_TRY(dev::launch_indexless_mark(st.a, static_cast<const uint64_t*>(st.off.p),
                                       static_cast<uint64_t*>(sub_abs.p), shift, ctx->stream));
    return Status::ok();
}

// HUFF_SYNC_DECODE=1: the one-pass index-free decoder (syncdec.hip) where it
// applies. Opt-in: measured slower than the pipeline (1 GiB
// Zipf 1.52-1.70 vs 1.04 ms; its look-back waits and variable-length output
// cost more than the second walk they save); the tests run both.
static bool sync_decode_enabled() {
    const char* e = std::getenv("HUFF_SYNC_DECODE");
    return e && *e == '1';
}

// The one-pass index-free decoder (syncdec.hip) into the caller's buffer.
// *done false: it does not apply, or it reported that its tail job list
// overflowed (pathologically skewed streams): the pipeline decodes instead.
static Status decode_sync(huff_ctx* ctx, const uint8_t* d_comp, uint64_t comp_bytes, uint64_t valid_bits,
                          const huff_tree* t, const DecTables* dt, uint8_t* d_user, size_t user_cap, bool* done,
                          uint64_t* nsym) {
    *done = false;
    if (!sync_decode_enabled() || dt->maxdepth > dt->sbits || dt->sbits < 1 || dt->sbits > 12) return Status::ok();
    uint32_t g = 0, lo_, hi_;
    t->t.depth_range(&lo_, &hi_, &g);
    if (g == 0) g = 1;
    // segments holding ~0.72 kSyncCap letters at the tree's Kraft mean, at an
    // odd dword stride (S = 32 mod 64: lanes start on different LDS banks),
    // a multiple of the gcd of the code lengths (every start in phase)
    const double target = 0.72 * dev::kSyncCap * dt->kraft_bits;
    uint64_t kmax = std::max<uint64_t>(1, static_cast<uint64_t>(target) / g);
    uint64_t S = g * kmax;
    for (uint64_t k = kmax; k >= 1 && k + 64 >= kmax; --k)
        if ((g * k) % 64 == 32) {
            S = g * k;
            break;
        }
    // lead-ins (HUFF_SYNC_LEAD / _LEAD0 for A/B): every lane's, and the
    // longer one of a tile's first lane
    auto env_u = [](const char* k, uint32_t d) {
        const char* e = std::getenv(k);
        return e && *e ? static_cast<uint32_t>(std::strtoul(e, nullptr, 10)) : d;
    };
    const uint32_t lead = std::max<uint32_t>(g, env_u("HUFF_SYNC_LEAD", 96) / g * g);
    const uint32_t lead0 = std::max<uint32_t>(lead, env_u("HUFF_SYNC_LEAD0", 256) / g * g);
    S = std::min<uint64_t>(std::max<uint64_t>(S, lead0), 1024 / g * g);
    const uint64_t nseg = (valid_bits + S - 1) / S;
    const uint64_t ntiles = (nseg + 255) / 256;
    if (ntiles > 0x7FFFFFFFull) return Status::ok();
    HUFF_TRY(ctx->sd_ws.ensure(32 + ntiles * 8));
    const uint64_t job_cap = nseg / 8 + 1024;
    HUFF_TRY(ctx->sd_jobs.ensure(job_cap * 24));
    HUFF_TRY(ctx->pin_total.ensure(8));
    if (!ctx->pin_total_dev) {
        std::memset(ctx->pin_total.p, 0, 8);
        HIP_TRY(hipHostGetDevicePointer(&ctx->pin_total_dev, ctx->pin_total.p, 0));
    }
    ctx->total_seq = (ctx->total_seq % 0xFFFF) + 1;
    uint8_t* ws = static_cast<uint8_t*>(ctx->sd_ws.p);
    dev::SyncDecArgs a{};
    a.comp = d_comp;
    a.comp_bytes = comp_bytes;
    a.valid_bits = valid_bits;
    a.seg_bits = S;
    a.nseg = nseg;
    a.lead_bits = lead;
    a.lead0_bits = lead0;
    a.stab = reinterpret_cast<const uint16_t*>(static_cast<const uint32_t*>(ctx->d_lut.p) + dt->soff);
    a.stab_bits = dt->sbits;
    a.out = d_user;
    a.out_cap = user_cap;
    a.ctrl = reinterpret_cast<unsigned int*>(ws);
    a.total = reinterpret_cast<unsigned long long*>(ws + 16);
    a.tile = reinterpret_cast<unsigned long long*>(ws + 32);
    a.jobs = static_cast<uint64_t*>(ctx->sd_jobs.p);
    a.job_cap = job_cap;
    a.host_total = static_cast<unsigned long long*>(ctx->pin_total_dev);
    a.tag = ctx->total_seq;
#ifdef HUFF_STAMPS
    a.stamps = stamp_region(0);
#endif
    HIP_TRY(hipMemsetAsync(ws, 0, 32 + ntiles * 8, ctx->stream));
    HIP_TRY(dev::launch_sync_decode(a, ctx->stream));
    HIP_TRY(hipEventRecord(ctx->lut_free, ctx->stream));
    const uint64_t* hw = static_cast<const uint64_t*>(ctx->pin_total.p);
    SpinWait sw;
    for (;;) {
        const uint64_t v = __atomic_load_n(hw, __ATOMIC_ACQUIRE);
        if ((v >> 48) == a.tag) {
            const uint64_t n = v & dev::kSyncBad;
            if (std::getenv("HUFF_FIX_STATS")) {  // diagnostics: the tail's jobs (a synchronising copy)
                unsigned int c[4];
                HIP_TRY(hipMemcpyAsync(c, a.ctrl, sizeof c, hipMemcpyDeviceToHost, ctx->stream));
                HIP_TRY(hipStreamSynchronize(ctx->stream));
                std::fprintf(stderr, "huff sync decode: segments %llu of %llu bits, tail jobs %u, look-back waits %u, %s\n",
                             static_cast<unsigned long long>(nseg), static_cast<unsigned long long>(S), c[dev::kSyncJobs],
                             c[dev::kSyncMis],
                             n == dev::kSyncBad ? "fell back to the pipeline" : "done");
            }
            if (n == dev::kSyncBad) return Status::ok();  // the pipeline instead
            *nsym = n;
            *done = true;
            return Status::ok();
        }
        if (sw.check_due()) {
            const hipError_t q = hipStreamQuery(ctx->stream);
            if (q == hipSuccess && (__atomic_load_n(hw, __ATOMIC_ACQUIRE) >> 48) != a.tag)
                return Status::err(HUFF_E_HIP, "the one-pass index-free decode finished without publishing its count");
            if (q != hipSuccess && q != hipErrorNotReady) HIP_TRY(q);
        }
    }
}

Status decode_indexless_dev(huff_ctx* ctx, const uint8_t* d_comp, uint64_t comp_bytes, uint64_t valid_bits,
                            const huff_tree* t, DevBuf& out, uint64_t* nsym, uint8_t* d_user, size_t user_cap,
                            unsigned long long* d_end) {
    *nsym = 0;
    // the output goes to d_user when given (capacity checked once the count
    // is known), else into `out`
    auto out_ptr = [&](uint64_t need) -> Status {
        if (d_user) {
            if (need > user_cap) return Status::err(HUFF_E_BUFFER_TOO_SMALL, "output buffer too small");
            return Status::ok();
        }
        return out.ensure(need + 16);
    };
    auto out_at = [&]() { return d_user ? d_user : static_cast<uint8_t*>(out.p); };
    if (valid_bits == 0) return Status::ok();
    HUFF_TRY(ctx->activate());
    if (reinterpret_cast<uintptr_t>(d_comp) & 15) {
        // the staged kernels read the stream in 16-B pieces: a stream at any
        // other alignment (a tensor view) is copied once to an aligned buffer
        HUFF_TRY(ctx->d_comp_align.ensure(comp_bytes + 64));
        HIP_TRY(hipMemcpyAsync(ctx->d_comp_align.p, d_comp, comp_bytes, hipMemcpyDeviceToDevice, ctx->stream));
        d_comp = static_cast<const uint8_t*>(ctx->d_comp_align.p);
    }
    const DecTables* dt = nullptr;
    HUFF_TRY(ctx->upload_dec_tables(t, &dt));
    // the window end (d_end): `count` codes walked from a known boundary
    auto walk_end = [&](const uint64_t* start, uint64_t start_v, const uint64_t* count, uint64_t count_v,
                        bool packed = false) -> Status {
        if (!d_end) return Status::ok();
        dev::WalkEndArgs w{};
        w.start_packed = packed ? 1u : 0u;
        w.comp = d_comp;
        w.comp_bytes = comp_bytes;
        w.lut = static_cast<const uint32_t*>(ctx->d_lut.p);
        w.lut_bits = dt->bits;
        w.start = start;
        w.start_v = start_v;
        w.count = count;
        w.count_v = count_v;
        w.end = d_end;
        HIP_TRY(dev::launch_walk_end(w, ctx->stream));
        return Status::ok();
    };
    if (dt->all8 && !fixed8_disabled()) {  // every code 8 bits: one symbol per whole byte
        const uint64_t n = valid_bits / 8;
        *nsym = n;
        HUFF_TRY(walk_end(nullptr, 8 * n, nullptr, 0));
        HUFF_TRY(out_ptr(n));
        dev::BytemapArgs m{};
        m.src = d_comp;
        m.dst = out_at();
        m.n = n;
        for (int b = 0; b < 256; ++b) m.map[b] = static_cast<uint8_t>(dt->lut[b]);
        HIP_TRY(dev::launch_bytemap(m, ctx->stream));
        return Status::ok();
    }
    if (dt->maxdepth > dev::kLongMaxLen) {  // deep codes: one lane walks the stream (deep.hip)
        DevBuf& cnt = ctx->idx_sub_abs;
        HUFF_TRY(cnt.ensure(8));
        dev::DeepSerialArgs d{};
        d.comp = d_comp;
        d.comp_bytes = comp_bytes;
        d.valid_bits = valid_bits;
        d.lut = static_cast<const uint32_t*>(ctx->d_lut.p);
        d.lut_bits = dt->bits;
        d.out = d_user;
        d.cap = d_user ? user_cap : 0;
        d.count = static_cast<unsigned long long*>(cnt.p);
        d.end = d_end;
        HIP_TRY(dev::launch_decode_deep_serial(d, ctx->stream));  // counts (and writes, when d_user is given)
        uint64_t total = 0;
        HIP_TRY(hipMemcpyAsync(&total, cnt.p, 8, hipMemcpyDeviceToHost, ctx->stream));
        HUFF_TRY(ctx->sync());
        *nsym = total;
        HUFF_TRY(out_ptr(total));
        if (!d_user) {  // into `out`, now that its size is known
            d.out = static_cast<uint8_t*>(out.p);
            d.cap = total;
            HIP_TRY(dev::launch_decode_deep_serial(d, ctx->stream));
        }
        HIP_TRY(hipEventRecord(ctx->lut_free, ctx->stream));
        return Status::ok();
    }
    const uint32_t check = decode_check_mode();
    if (d_user && !d_end && !check) {  // one pass (syncdec.hip), when it applies
        bool done = false;
        HUFF_TRY(decode_sync(ctx, d_comp, comp_bytes, valid_bits, t, dt, d_user, user_cap, &done, nsym));
        if (done) return out_ptr(*nsym);  // (a short buffer: nothing past it was written)
    }
    IndexlessSync& st = ctx->indexless_ws();
    st.dt = dt;
    // with a caller's buffer, the marks go out before the host waits for the
    // count: sub_abs sized for the most symbols the stream or the buffer can
    // hold (shortest code), k_mark_lite bounded to it (22 us of idle stream
    // between the scan and k_mark_lite otherwise)
    bool marked = false;
    // the compact marks (u32 per 64 symbols + u32 per task: dev::mark32_*)
    // unless a consumer wants absolute u64 marks (the window end of the file
    // path, the check build)
    const bool compact = !check && !d_end;
    auto mark_early = [&]() -> Status {
        if (!d_user || check || d_end || !st.block_off || !dev::indexless_staged(st.a)) return Status::ok();
        uint32_t min_len = 64, max_len_;
        t->t.depth_range(&min_len, &max_len_);
        const uint64_t most = std::min<uint64_t>(user_cap, valid_bits / min_len);
        const uint64_t runs = (most + 63) >> 6;
        HUFF_TRY(ctx->idx_mark32.ensure(runs * 4 + 8));
        HUFF_TRY(ctx->idx_task_seg.ensure(((most + dev::kTaskSym - 1) / dev::kTaskSym) * 4 + 8));
        HIP_TRY(dev::launch_indexless_mark_lite(st.a, nullptr, static_cast<const unsigned long long*>(st.woff.p),
                                                nullptr, runs, ctx->stream, static_cast<uint32_t*>(ctx->idx_mark32.p),
                                                static_cast<uint32_t*>(ctx->idx_task_seg.p)));
        marked = true;
        return Status::ok();
    };
    // k_emit (codes > 32 bits) and the walked marks of the check build read every segment's offset
    HUFF_TRY(indexless_sync(ctx, d_comp, comp_bytes, valid_bits, t, st, check != 0, mark_early));
    const uint64_t total = st.total;
    *nsym = total;
    if (total == 0) HUFF_TRY(walk_end(nullptr, 0, nullptr, 0));
    HUFF_TRY(out_ptr(total));
    hipStream_t strm = ctx->stream;
    if (dev::indexless_staged(st.a) && total && !(reinterpret_cast<uintptr_t>(d_comp) & 15)) {
        // a misaligned output: decoded into an aligned buffer, then copied (as huff_enc::decode)
        const bool bounce = reinterpret_cast<uintptr_t>(out_at()) & 15;
        if (bounce) HUFF_TRY(ctx->d_align.ensure(total + 64));
        // a restart point every 64 symbols, then the fixed-count decoder
        // (k_mark_lite: a boundary and the codes to skip from it, the
        // decoder's lanes walk those codes themselves; the self-check builds,
        // HUFF_DEC_VARIANT=11, needs exact lane starts: k_mark_lds walks)
        DevBuf& sub_abs = ctx->idx_sub_abs;
        if (check) {
            HUFF_TRY(indexless_mark(ctx, st, sub_abs, 6));
        } else if (!marked && compact) {
            HUFF_TRY(ctx->idx_mark32.ensure(((total + 63) >> 6) * 4 + 8));
            HUFF_TRY(ctx->idx_task_seg.ensure(((total + dev::kTaskSym - 1) / dev::kTaskSym) * 4 + 8));
            HIP_TRY(dev::launch_indexless_mark_lite(
                st.a, st.block_off ? nullptr : static_cast<const uint64_t*>(st.off.p),
                st.block_off ? static_cast<const unsigned long long*>(st.woff.p) : nullptr, nullptr, ~0ull, strm,
                static_cast<uint32_t*>(ctx->idx_mark32.p), static_cast<uint32_t*>(ctx->idx_task_seg.p)));
        } else if (!marked) {
            HUFF_TRY(sub_abs.ensure(((total + 63) >> 6) * 8 + 8));
            HIP_TRY(dev::launch_indexless_mark_lite(
                st.a, st.block_off ? nullptr : static_cast<const uint64_t*>(st.off.p),
                st.block_off ? static_cast<const unsigned long long*>(st.woff.p) : nullptr,
                static_cast<uint64_t*>(sub_abs.p), ~0ull, strm));
        }
        const uint64_t m = ((total - 1) >> 6) << 6;  // the last mark: symbol m
        if (!compact)  // (d_end never goes with the compact marks)
            HUFF_TRY(walk_end(static_cast<const uint64_t*>(sub_abs.p) + (m >> 6), 0, nullptr, total - m, !check));
        dev::DecodeArgs d{};
        d.comp = d_comp;
        d.comp_bytes = comp_bytes;
        d.lut = static_cast<const uint32_t*>(ctx->d_lut.p);
        d.lut_bits = dt->bits;
        d.lut_words = static_cast<uint32_t>(dt->lut.size());
        d.sub_abs64 = compact ? nullptr : static_cast<const uint64_t*>(sub_abs.p);
        d.mark32 = compact ? static_cast<const uint32_t*>(ctx->idx_mark32.p) : nullptr;
        d.task_seg = compact ? static_cast<const uint32_t*>(ctx->idx_task_seg.p) : nullptr;
        d.seg_bits = static_cast<uint32_t>(st.a.seg_bits);
        d.skip_packed = check ? 0u : 1u;
        d.end_bit = valid_bits;
        d.nchunks = static_cast<uint32_t>((total + dev::kChunk - 1) / dev::kChunk);
        d.max_len = dt->maxdepth;
        d.stab = reinterpret_cast<const uint16_t*>(static_cast<const uint32_t*>(ctx->d_lut.p) + dt->soff);
        d.stab_bits = dt->sbits;
        d.cu_count = static_cast<uint32_t>(ctx->cu_count);
        d.pad_stage = dev::fixed_decode_pad(valid_bits, total);
        d.small_stage = small_stage_enabled() && dev::fixed_decode_small(valid_bits, total);
        d.dma_stage = dma_decode_enabled();
        d.n = total;
        d.out = bounce ? static_cast<uint8_t*>(ctx->d_align.p) : out_at();
        d.check_mode = check;
        HUFF_TRY(run_checked_decode(ctx, d, [&] { return dev::launch_decode_fixed(d, strm); }));
        HIP_TRY(hipEventRecord(ctx->lut_free, strm));
        if (bounce) HIP_TRY(hipMemcpyAsync(out_at(), ctx->d_align.p, total, hipMemcpyDeviceToDevice, strm));
        return Status::ok();
    }
    HIP_TRY(dev::launch_indexless_emit(st.a, static_cast<const uint64_t*>(st.off.p), out_at(), strm));
    if (total)  // the last segment's codes from its settled start
        HUFF_TRY(walk_end(st.a.s + st.a.nseg - 1, 0, st.a.c + st.a.nseg - 1, 0));
    HIP_TRY(hipEventRecord(ctx->lut_free, strm));
    return Status::ok();
}

Status decode_indexless_host(huff_ctx* ctx, const uint8_t* comp, size_t len, uint64_t valid_bits, const huff_tree* t,
                             std::vector<uint8_t>& out) {
    out.clear();
    HUFF_TRY(ctx->activate());
    DevBuf d_comp, d_out;
    HUFF_TRY(d_comp.ensure(len + 16));
    HIP_TRY(hipMemcpyAsync(d_comp.p, comp, len, hipMemcpyHostToDevice, ctx->stream));
    uint64_t n = 0;
    HUFF_TRY(decode_indexless_dev(ctx, static_cast<const uint8_t*>(d_comp.p), len, valid_bits, t, d_out, &n));
    out.resize(n);
    if (n) HIP_TRY(hipMemcpyAsync(out.data(), d_out.p, n, hipMemcpyDeviceToHost, ctx->stream));
    return ctx->sync();
}

}  // namespace huff

#ifdef HUFF_STAMPS
// timing builds only: region r's first `words` stamp words into host memory
extern "C" int huff_diag_stamps(int r, uint64_t* host, size_t words) {
    uint64_t* p = huff::stamp_region(r);
    if (!p || words > huff::kStampRegionWords) return -1;
    return hipMemcpy(host, p, words * 8, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
