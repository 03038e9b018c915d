// comm_rccl.hip -- a library-owned RCCL communicator behind npgx_comm (the
// collectives of the exactly-sharded AnchorFinder and block build, SURVEY.md
// §8e, DESIGN.md "Multi-GPU").
//
// One process per GPU.  Rank 0 makes the RCCL unique id (npgx_rccl_unique_id)
// and the launcher hands it to every rank (the bench passes it through
// torch.distributed's object broadcast); each rank then opens its
// communicator on its own device with npgx_rccl_comm_create.  The collectives
// run on the communicator's stream over xGMI, device buffers in and out, no
// host staging:
//   allreduce_i32  -> ncclAllReduce (SUM / MIN) in place;
//   allgather_i64  -> ncclAllGather of one int64 per rank (then to the host);
//   allgatherv_u64 -> one ncclBroadcast per rank with a non-empty part, in a
//                     group, each straight into its place in the output.
// The library calls a collective with its own stream idle and expects the data
// in place when the call returns, so each call ends with a stream wait.
#include <rccl/rccl.h>

#include <cstring>

#include "common.hpp"

namespace npgx {

struct RcclState {
    ncclComm_t comm = nullptr;
    hipStream_t stream = nullptr;
    int device = 0;
    DevBuf<int64_t> one, all;  // allgather_i64 staging (1 and world values)
};

static int rccl_ok(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return 0;
    set_last_error(std::string(what) + ": " + ncclGetErrorString(r));
    return -1;
}

extern "C" {
static int cb_allreduce_i32(void* user, int32_t* dev, int64_t n, int32_t op) {
    RcclState* S = (RcclState*)user;
    if (n == 0) return 0;
    DeviceGuard dg(S->device);
    if (!dg.ok) return -1;
    if (rccl_ok(ncclAllReduce(dev, dev, (size_t)n, ncclInt32, op == NPGX_OP_MIN ? ncclMin : ncclSum, S->comm,
                              S->stream),
                "ncclAllReduce"))
        return -1;
    return stream_wait(S->stream) == hipSuccess ? 0 : -1;
}

static int cb_allgather_i64(void* user, int64_t value, int64_t* out) {
    RcclState* S = (RcclState*)user;
    int world = 0;
    DeviceGuard dg(S->device);
    if (!dg.ok) return -1;
    if (rccl_ok(ncclCommCount(S->comm, &world), "ncclCommCount")) return -1;
    if (hipMemcpyAsync(S->one.p, &value, 8, hipMemcpyHostToDevice, S->stream) != hipSuccess) return -1;
    if (rccl_ok(ncclAllGather(S->one.p, S->all.p, 1, ncclInt64, S->comm, S->stream), "ncclAllGather")) return -1;
    if (hipMemcpyAsync(out, S->all.p, (size_t)world * 8, hipMemcpyDeviceToHost, S->stream) != hipSuccess) return -1;
    return stream_wait(S->stream) == hipSuccess ? 0 : -1;
}

static int cb_allgatherv_u64(void* user, const uint64_t* dev_in, const int64_t* counts, uint64_t* dev_out) {
    RcclState* S = (RcclState*)user;
    int world = 0, rank = 0;
    DeviceGuard dg(S->device);
    if (!dg.ok) return -1;
    if (rccl_ok(ncclCommCount(S->comm, &world), "ncclCommCount")) return -1;
    if (rccl_ok(ncclCommUserRank(S->comm, &rank), "ncclCommUserRank")) return -1;
    if (rccl_ok(ncclGroupStart(), "ncclGroupStart")) return -1;
    int64_t off = 0;
    for (int r = 0; r < world; r++) {
        if (counts[r] > 0 &&
            rccl_ok(ncclBroadcast(r == rank ? (const void*)dev_in : (const void*)(dev_out + off), dev_out + off,
                                  (size_t)counts[r], ncclUint64, r, S->comm, S->stream),
                    "ncclBroadcast")) {
            ncclGroupEnd();
            return -1;
        }
        off += counts[r];
    }
    if (rccl_ok(ncclGroupEnd(), "ncclGroupEnd")) return -1;
    return stream_wait(S->stream) == hipSuccess ? 0 : -1;
}
}  // extern "C"

}  // namespace npgx

using namespace npgx;

extern "C" {

int npgx_rccl_unique_id(void* out) {
    return guard([&] {
        NPGX_REQUIRE(out, NPGX_ERR_ARG, "null argument");
        static_assert(sizeof(ncclUniqueId) == NPGX_RCCL_ID_BYTES, "RCCL unique id size");
        ncclUniqueId id;
        const ncclResult_t r = ncclGetUniqueId(&id);
        NPGX_REQUIRE(r == ncclSuccess, NPGX_ERR_HIP, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
        memcpy(out, &id, sizeof(id));
    });
}

int npgx_rccl_comm_create(const void* unique_id, int32_t rank, int32_t world, int32_t device, npgx_comm** out) {
    return guard([&] {
        NPGX_REQUIRE(unique_id && out, NPGX_ERR_ARG, "null argument");
        NPGX_REQUIRE(world >= 1 && rank >= 0 && rank < world, NPGX_ERR_ARG, "bad rank / world");
        DeviceGuard dg(device);
        NPGX_REQUIRE(dg.ok, NPGX_ERR_HIP, "hipSetDevice failed");
        auto* S = new RcclState;
        S->device = device;
        try {
            NPGX_HIP(hipStreamCreateWithFlags(&S->stream, hipStreamNonBlocking));
            ncclUniqueId id;
            memcpy(&id, unique_id, sizeof(id));
            const ncclResult_t r = ncclCommInitRank(&S->comm, world, id, rank);
            NPGX_REQUIRE(r == ncclSuccess, NPGX_ERR_HIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
            S->one.ensure(1);
            S->all.ensure((size_t)world);
        } catch (...) {
            if (S->comm) ncclCommDestroy(S->comm);
            if (S->stream) (void)hipStreamDestroy(S->stream);
            delete S;
            throw;
        }
        auto* c = new npgx_comm;
        c->rank = rank;
        c->world = world;
        c->user = S;
        c->allreduce_i32 = cb_allreduce_i32;
        c->allgather_i64 = cb_allgather_i64;
        c->allgatherv_u64 = cb_allgatherv_u64;
        *out = c;
    });
}

int npgx_rccl_comm_count(const npgx_comm* c, int32_t* n) {
    return guard([&] {
        NPGX_REQUIRE(c && c->user && n, NPGX_ERR_ARG, "null argument");
        auto* S = (RcclState*)c->user;
        int w = 0;
        const ncclResult_t r = ncclCommCount(S->comm, &w);
        NPGX_REQUIRE(r == ncclSuccess, NPGX_ERR_HIP, std::string("ncclCommCount: ") + ncclGetErrorString(r));
        *n = w;
    });
}

int npgx_comm_check(const npgx_comm* c) {
    return guard([&] {
        NPGX_REQUIRE(c && c->allreduce_i32 && c->allgather_i64 && c->allgatherv_u64, NPGX_ERR_ARG,
                     "null argument");
        const int W = c->world, R = c->rank;
        NPGX_REQUIRE(W >= 1 && R >= 0 && R < W, NPGX_ERR_ARG, "bad rank / world");
        // allreduce SUM / MIN of (rank + 1 + i) over 1000 values
        const int64_t n = 1000;
        std::vector<int32_t> h((size_t)n);
        DevBuf<int32_t> d;
        d.ensure((size_t)n);
        for (int op = 0; op < 2; op++) {
            for (int64_t i = 0; i < n; i++) h[(size_t)i] = R + 1 + (int32_t)i;
            NPGX_HIP(hipMemcpy(d.p, h.data(), (size_t)n * 4, hipMemcpyHostToDevice));
            NPGX_REQUIRE(c->allreduce_i32(c->user, d.p, n, op == 0 ? NPGX_OP_SUM : NPGX_OP_MIN) == 0, NPGX_ERR_HIP,
                         "allreduce_i32 failed");
            NPGX_HIP(hipMemcpy(h.data(), d.p, (size_t)n * 4, hipMemcpyDeviceToHost));
            for (int64_t i = 0; i < n; i++) {
                const int32_t want = op == 0 ? (int32_t)(W * (W + 1) / 2 + W * i) : (int32_t)(1 + i);
                NPGX_REQUIRE(h[(size_t)i] == want, NPGX_ERR_STATE, "allreduce_i32 gave a wrong value");
            }
        }
        // allgather_i64 of 1000 * rank + 7
        std::vector<int64_t> g((size_t)W);
        NPGX_REQUIRE(c->allgather_i64(c->user, 1000 * (int64_t)R + 7, g.data()) == 0, NPGX_ERR_HIP,
                     "allgather_i64 failed");
        for (int r = 0; r < W; r++)
            NPGX_REQUIRE(g[(size_t)r] == 1000 * (int64_t)r + 7, NPGX_ERR_STATE, "allgather_i64 gave a wrong value");
        // allgatherv_u64: rank r sends (r + 1) % 3 * 1000 values (every third empty), value = r << 32 | i
        std::vector<int64_t> cnt((size_t)W);
        int64_t tot = 0;
        for (int r = 0; r < W; r++) tot += (cnt[(size_t)r] = ((r + 1) % 3) * 1000);
        std::vector<uint64_t> mine((size_t)std::max<int64_t>(cnt[(size_t)R], 1));
        for (int64_t i = 0; i < cnt[(size_t)R]; i++) mine[(size_t)i] = ((uint64_t)R << 32) | (uint64_t)i;
        DevBuf<uint64_t> din, dout;
        din.ensure(mine.size());
        dout.ensure((size_t)std::max<int64_t>(tot, 1));
        NPGX_HIP(hipMemcpy(din.p, mine.data(), mine.size() * 8, hipMemcpyHostToDevice));
        NPGX_REQUIRE(c->allgatherv_u64(c->user, din.p, cnt.data(), dout.p) == 0, NPGX_ERR_HIP, "allgatherv_u64 failed");
        std::vector<uint64_t> all((size_t)std::max<int64_t>(tot, 1));
        NPGX_HIP(hipMemcpy(all.data(), dout.p, (size_t)tot * 8, hipMemcpyDeviceToHost));
        int64_t k = 0;
        for (int r = 0; r < W; r++)
            for (int64_t i = 0; i < cnt[(size_t)r]; i++, k++)
                NPGX_REQUIRE(all[(size_t)k] == (((uint64_t)r << 32) | (uint64_t)i), NPGX_ERR_STATE,
                             "allgatherv_u64 gave a wrong value");
    });
}

void npgx_rccl_comm_free(npgx_comm* c) {
    if (!c) return;
    auto* S = (RcclState*)c->user;
    if (S) {
        DeviceGuard dg(S->device);
        if (S->comm) ncclCommDestroy(S->comm);
        if (S->stream) (void)hipStreamDestroy(S->stream);
        delete S;
    }
    delete c;
}

}  // extern "C"
