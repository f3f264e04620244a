// mgpu.cpp — multi-GPU sharded compress behind the C ABI.
//
// One process (or thread) per GPU, each with its own huff_ctx. A huff_comm is
// an RCCL communicator over xGMI owned next to the context: the caller makes
// a unique id on rank 0 (huff_comm_unique_id), hands its 128 bytes to every
// rank over any channel it has (MPI, TCP, a file), and each rank joins with
// huff_comm_init. huff_mgpu_compress then runs the whole sharded encode of
// the rank's job in one call (huff_mgpu_pack_rows is its host half, for
// callers that exchange the rows over their own channel;
// huff_mgpu_exchange_launch queues the exchange of the next call ahead):
//
//   pass 1 (hist256 + row kernel)  -> ncclAllGather of a 258 x int64 row per
//   rank on the context stream     -> one device-to-host copy, ONE host wait
//   -> host tree of the summed weights (identical on every rank)
//   -> this rank's bit base = sum of the previous ranks' bits, its shared
//      first byte completed from the previous ranks' tail bytes -> pass 2.
//
// This replaces the reference's weights merge (huff/src/comp.rs:161-172,
// weights.rs:293-319: ByteWeights of the whole input = the sum of the
// per-part weights) with one collective; the all-gather (not an all-reduce)
// also gives every rank every rank's bit count, so no second collective
// computes the bit bases. Messages are 2 KiB per rank: latency-bound.
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <memory>
#include <vector>

#include "../capi_util.hpp"
#include "runtime.hpp"
#include "huffgpu.h"

using huff::capi::fail;
using huff::capi::guarded;

struct huff_comm {
    huff_ctx* ctx = nullptr;
    ncclComm_t comm = nullptr;
    int world = 0, rank = 0;
    DevBuf row, rows;    // this rank's row, the gathered rows (device)
    PinnedBuf host_rows; // the gathered rows (host); its event follows their copy
    // an exchange queued ahead by huff_mgpu_exchange_launch for this job, not
    // yet consumed by huff_mgpu_compress, and the job's own pass-1 status
    const huff_enc* pending = nullptr;
    huff::Status pending_local;
    ~huff_comm() {
        if (comm) ncclCommDestroy(comm);
    }
};

namespace {

huff::Status nccl_status(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return huff::Status::ok();
    return huff::Status::err(HUFF_E_HIP, std::string(what) + ": " + ncclGetErrorString(r));
}
#define NCCL_TRY(expr) HUFF_TRY(nccl_status((expr), #expr))

constexpr size_t kRowWords = 258;  // huff_enc_hist_row: 256 weights, tail bytes, tail count

}  // namespace

extern "C" {

int huff_comm_unique_id(uint8_t id[HUFF_COMM_ID_BYTES]) {
    if (!id) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&]() -> huff::Status {
        static_assert(sizeof(ncclUniqueId) == HUFF_COMM_ID_BYTES, "RCCL unique id size");
        ncclUniqueId u;
        NCCL_TRY(ncclGetUniqueId(&u));
        std::memcpy(id, &u, sizeof u);
        return huff::Status::ok();
    });
}

int huff_comm_init(huff_ctx* ctx, const uint8_t id[HUFF_COMM_ID_BYTES], int world, int rank, huff_comm** out) {
    if (!ctx || !id || !out || world < 1 || rank < 0 || rank >= world)
        return fail(HUFF_E_INVALID_ARG, "null or out-of-range argument");
    *out = nullptr;
    return guarded([&]() -> huff::Status {
        HUFF_TRY(ctx->activate());
        auto c = std::make_unique<huff_comm>();
        c->ctx = ctx;
        c->world = world;
        c->rank = rank;
        ncclUniqueId u;
        std::memcpy(&u, id, sizeof u);
        NCCL_TRY(ncclCommInitRank(&c->comm, world, u, rank));
        HUFF_TRY(c->row.ensure(kRowWords * 8));
        HUFF_TRY(c->rows.ensure(kRowWords * 8 * static_cast<size_t>(world)));
        HUFF_TRY(c->host_rows.ensure(kRowWords * 8 * static_cast<size_t>(world)));
        *out = c.release();
        return huff::Status::ok();
    });
}

void huff_comm_free(huff_comm* c) { delete c; }

// The world the communicator itself reports (ncclCommCount /
// ncclCommUserRank), not the arguments it was created with: a bench line can
// then prove how many ranks RCCL joined (huff/src/comp.rs:161-172 is the
// merge this communicator replaces).
int huff_comm_world(const huff_comm* c, int* world, int* rank) {
    if (!c || !world || !rank) return fail(HUFF_E_INVALID_ARG, "null argument");
    return guarded([&]() -> huff::Status {
        int n = 0, r = 0;
        NCCL_TRY(ncclCommCount(c->comm, &n));
        NCCL_TRY(ncclCommUserRank(c->comm, &r));
        if (n != c->world || r != c->rank)
            return huff::Status::err(HUFF_E_HIP, "RCCL reports world " + std::to_string(n) + " rank " +
                                                     std::to_string(r) + ", created as world " +
                                                     std::to_string(c->world) + " rank " + std::to_string(c->rank));
        *world = n;
        *rank = r;
        return huff::Status::ok();
    });
}

int huff_mgpu_pack_rows(huff_enc* e, const int64_t* rows, int world, int rank, uint8_t* d_out, size_t out_cap,
                        huff_tree** tree_out, uint64_t* bit_base_out, uint64_t* bits_out,
                        uint64_t* owned_bytes_out) {
    if (!e || !rows || !d_out || !tree_out || world < 1 || rank < 0 || rank >= world)
        return fail(HUFF_E_INVALID_ARG, "null or out-of-range argument");
    if (reinterpret_cast<uintptr_t>(d_out) & 15) return fail(HUFF_E_INVALID_ARG, "d_out must be 16-byte aligned");
    *tree_out = nullptr;
    return guarded([&]() -> huff::Status {
        const size_t W = static_cast<size_t>(world);
        std::vector<uint64_t> hists(W * 256);
        std::vector<uint8_t> tails(W * 8), tail_lens(W);
        for (size_t q = 0; q < W; ++q) {
            const int64_t tl = rows[q * kRowWords + 257];
            if (tl < 0) return huff::Status::err(HUFF_E_INVALID_ARG, "rank " + std::to_string(q) +
                                                 " failed before the exchange");
            if (tl > 8) return huff::Status::err(HUFF_E_INVALID_ARG, "malformed row: tail count > 8");
            std::memcpy(&hists[q * 256], rows + q * kRowWords, 256 * 8);
            std::memcpy(&tails[q * 8], rows + q * kRowWords + 256, 8);  // little-endian: stream order
            tail_lens[q] = static_cast<uint8_t>(tl);
        }
        uint64_t base = 0, bits = 0;
        huff_tree* t = nullptr;
        const int rc = huff_enc_pack_shards(e, hists.data(), static_cast<uint32_t>(world), static_cast<uint32_t>(rank),
                                            tails.data(), tail_lens.data(), d_out, out_cap, &t, &base, &bits);
        if (bit_base_out) *bit_base_out = base;
        if (bits_out) *bits_out = bits;
        if (rc != HUFF_OK) return huff::Status::err(rc, huff::capi::last_error());
        // the rank owns its first (shared) byte and leaves its partial last
        // byte to the next rank, except the last rank (mgpu.owned_bytes)
        const uint64_t end = (base & 7) + bits;
        if (owned_bytes_out) *owned_bytes_out = rank + 1 == world ? (end + 7) / 8 : end / 8;
        *tree_out = t;
        return huff::Status::ok();
    });
}

namespace {

// pass 1 -> row -> all-gather -> rows to pinned host memory, all queued on
// the context stream (the copy's completion recorded on host_rows.ev). A
// rank that cannot run its pass 1 still takes part in the collective, with a
// row that marks it failed (tail count -1): every rank then returns an error
// instead of the others blocking in ncclAllGather. The local failure (its
// own status code: argument, HIP, memory) is returned in *local.
huff::Status queue_exchange(huff_comm* c, huff_enc* e, huff::Status* local) {
    huff_ctx* ctx = c->ctx;
    // a context that cannot be activated cannot post its row either: the
    // other ranks would block in the collective, so say so loudly
    HUFF_TRY(ctx->activate());
    const size_t world = static_cast<size_t>(c->world);
    if (!*local) *local = e->hist_row(static_cast<long long*>(c->row.p));
    if (*local) {
        static const std::vector<int64_t> bad = [] {
            std::vector<int64_t> r(kRowWords, 0);
            r[257] = -1;
            return r;
        }();
        HIP_TRY_RT(hipMemcpyAsync(c->row.p, bad.data(), kRowWords * 8, hipMemcpyHostToDevice, ctx->stream));
    }
    NCCL_TRY(ncclAllGather(c->row.p, c->rows.p, kRowWords, ncclInt64, c->comm, ctx->stream));
    HIP_TRY_RT(hipMemcpyAsync(c->host_rows.p, c->rows.p, kRowWords * 8 * world, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY_RT(hipEventRecord(c->host_rows.ev, ctx->stream));
    return huff::Status::ok();
}

}  // namespace

// The exchange of the job's next compress queued now (a streaming encoder's
// software pipeline: queued between a pack and its decode, the wait and tree
// of the next huff_mgpu_compress overlap that decode). Every rank must queue
// it at the same point of its stream order, as for any collective.
int huff_mgpu_exchange_launch(huff_comm* c, huff_enc* e) {
    if (!c) return fail(HUFF_E_INVALID_ARG, "null communicator");
    if (c->pending)  // no collective queued: every rank fails the same way
        return fail(HUFF_E_STATE, "an exchange is already pending on this communicator");
    huff::Status local;
    if (!e) local = huff::Status::err(HUFF_E_INVALID_ARG, "null argument");
    else if (e->ctx != c->ctx) local = huff::Status::err(HUFF_E_INVALID_ARG, "a job of another context");
    return guarded([&]() -> huff::Status {
        HUFF_TRY(queue_exchange(c, e, &local));
        c->pending = e;
        c->pending_local = local;
        return huff::Status::ok();
    });
}

int huff_mgpu_compress(huff_comm* c, huff_enc* e, uint8_t* d_out, size_t out_cap, huff_tree** tree_out,
                       uint64_t* bit_base_out, uint64_t* bits_out, uint64_t* owned_bytes_out) {
    if (!c) return fail(HUFF_E_INVALID_ARG, "null communicator");
    if (tree_out) *tree_out = nullptr;
    if (c->pending && c->pending != e)
        return fail(HUFF_E_STATE, "an exchange of another job is pending on this communicator");
    huff::Status local;
    if (!e || !d_out || !tree_out) local = huff::Status::err(HUFF_E_INVALID_ARG, "null argument");
    else if (e->ctx != c->ctx) local = huff::Status::err(HUFF_E_INVALID_ARG, "a job of another context");
    else if (reinterpret_cast<uintptr_t>(d_out) & 15)
        local = huff::Status::err(HUFF_E_INVALID_ARG, "d_out must be 16-byte aligned");
    return guarded([&]() -> huff::Status {
        if (c->pending) {  // queued ahead: only the wait is left
            c->pending = nullptr;
            if (!local) local = c->pending_local;
        } else {
            HUFF_TRY(queue_exchange(c, e, &local));
        }
        HUFF_TRY(c->host_rows.wait());  // the rows' copy, not the work queued after it
        if (local) return local;
        const int rc = huff_mgpu_pack_rows(e, static_cast<const int64_t*>(c->host_rows.p), c->world, c->rank, d_out,
                                           out_cap, tree_out, bit_base_out, bits_out, owned_bytes_out);
        if (rc != HUFF_OK) return huff::Status::err(rc, huff::capi::last_error());
        return huff::Status::ok();
    });
}

}  // extern "C"
