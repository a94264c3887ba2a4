// a12-a14 at the C ABI: the learner's collectives as RCCL calls over xGMI, for hosts that bind
// the library directly (skyrl_comm_{init, allreduce, broadcast}). The Python
// host (skyrl_amd/comm.py) reaches the same RCCL through torch.distributed; skyrl_amd/rccl.py
// binds these entry points.
//
// Reference call sites they stand in for (skyrl-train/skyrl_train/):
//   all-reduce      metric reduction, distributed/strategy.py:70-95 (one call per scalar there)
//                   and the DP gradient mean, distributed/fsdp_strategy.py:216-226
//   reduce-scatter  FSDP2's fp32 gradient reduce-scatter, distributed/fsdp_strategy.py:253-271
//   all-gather      FSDP2's parameter all-gather (the sharded optimizer's bf16 / fp32 shards)
//   broadcast       learner -> rollout weights, weight_sync/broadcast_strategy.py:98-191
//
// One communicator per process and GPU (the current HIP device at init). Every call is
// stream-ordered on the caller's hipStream_t, never synchronizes the host and allocates nothing.
// The communicator handle is caller-owned (no global state): init / destroy bracket its life.
#include "common.h"

#include <rccl/rccl.h>

namespace skyrl {
namespace {

int nccl_fail(const char* what, ncclResult_t r) {
    return fail(SKYRL_ERR_LAUNCH, std::string(what) + ": " + ncclGetErrorString(r));
}

bool nccl_type(int dtype, ncclDataType_t& t) {
    switch (dtype) {
        case SKYRL_F32: t = ncclFloat32; return true;
        case SKYRL_BF16: t = ncclBfloat16; return true;
        case SKYRL_I64: t = ncclInt64; return true;
        case SKYRL_I32: t = ncclInt32; return true;
        case SKYRL_U8: t = ncclUint8; return true;
        default: return false;
    }
}

bool nccl_op(int op, ncclRedOp_t& o) {
    switch (op) {
        case SKYRL_COMM_SUM: o = ncclSum; return true;
        case SKYRL_COMM_MAX: o = ncclMax; return true;
        case SKYRL_COMM_MIN: o = ncclMin; return true;
        case SKYRL_COMM_AVG: o = ncclAvg; return true;
        default: return false;
    }
}

}  // namespace
}  // namespace skyrl

using namespace skyrl;

extern "C" size_t skyrl_comm_unique_id_bytes(void) { return sizeof(ncclUniqueId); }

extern "C" int skyrl_comm_get_unique_id(void* id_out) {
    SKYRL_REQUIRE(id_out, "comm_get_unique_id: null pointer");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) return nccl_fail("ncclGetUniqueId", r);
    __builtin_memcpy(id_out, &id, sizeof(id));
    return SKYRL_OK;
}

extern "C" int skyrl_comm_init(const void* unique_id, int32_t nranks, int32_t rank, void** comm_out) {
    SKYRL_REQUIRE(unique_id && comm_out, "comm_init: null pointer");
    SKYRL_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "comm_init: rank must be in [0, nranks)");
    ncclUniqueId id;
    __builtin_memcpy(&id, unique_id, sizeof(id));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = ncclCommInitRank(&comm, nranks, id, rank);
    if (r != ncclSuccess) return nccl_fail("ncclCommInitRank", r);
    *comm_out = comm;
    return SKYRL_OK;
}

extern "C" int skyrl_comm_destroy(void* comm) {
    if (!comm) return SKYRL_OK;
    const ncclResult_t r = ncclCommDestroy(reinterpret_cast<ncclComm_t>(comm));
    return r == ncclSuccess ? SKYRL_OK : nccl_fail("ncclCommDestroy", r);
}

extern "C" int skyrl_comm_size(void* comm, int32_t* nranks_out, int32_t* rank_out) {
    SKYRL_REQUIRE(comm && nranks_out && rank_out, "comm_size: null pointer");
    int n = 0, r = 0;
    ncclResult_t e = ncclCommCount(reinterpret_cast<ncclComm_t>(comm), &n);
    if (e == ncclSuccess) e = ncclCommUserRank(reinterpret_cast<ncclComm_t>(comm), &r);
    if (e != ncclSuccess) return nccl_fail("ncclCommCount", e);
    *nranks_out = n;
    *rank_out = r;
    return SKYRL_OK;
}

#define SKYRL_COMM_ARGS(what)                                                        \
    SKYRL_REQUIRE(comm, what ": null communicator");                                 \
    ncclDataType_t t;                                                                \
    SKYRL_REQUIRE(nccl_type(dtype, t), what ": dtype must be one of SKYRL_F32 .. SKYRL_U8")

extern "C" int skyrl_comm_allreduce(const void* send, void* recv, int64_t count, int dtype, int op, void* comm,
                                    void* stream) {
    SKYRL_COMM_ARGS("comm_allreduce");
    ncclRedOp_t o;
    SKYRL_REQUIRE(nccl_op(op, o), "comm_allreduce: op must be SKYRL_COMM_SUM/MAX/MIN/AVG");
    SKYRL_REQUIRE(count >= 0 && (count == 0 || (send && recv)), "comm_allreduce: bad buffers");
    const ncclResult_t r = ncclAllReduce(send, recv, (size_t)count, t, o, reinterpret_cast<ncclComm_t>(comm),
                                         as_stream(stream));
    return r == ncclSuccess ? SKYRL_OK : nccl_fail("ncclAllReduce", r);
}

extern "C" int skyrl_comm_reduce_scatter(const void* send, void* recv, int64_t recv_count, int dtype, int op,
                                         void* comm, void* stream) {
    SKYRL_COMM_ARGS("comm_reduce_scatter");
    ncclRedOp_t o;
    SKYRL_REQUIRE(nccl_op(op, o), "comm_reduce_scatter: op must be SKYRL_COMM_SUM/MAX/MIN/AVG");
    SKYRL_REQUIRE(recv_count >= 0 && (recv_count == 0 || (send && recv)), "comm_reduce_scatter: bad buffers");
    const ncclResult_t r = ncclReduceScatter(send, recv, (size_t)recv_count, t, o, reinterpret_cast<ncclComm_t>(comm),
                                             as_stream(stream));
    return r == ncclSuccess ? SKYRL_OK : nccl_fail("ncclReduceScatter", r);
}

extern "C" int skyrl_comm_allgather(const void* send, void* recv, int64_t send_count, int dtype, void* comm,
                                    void* stream) {
    SKYRL_COMM_ARGS("comm_allgather");
    SKYRL_REQUIRE(send_count >= 0 && (send_count == 0 || (send && recv)), "comm_allgather: bad buffers");
    const ncclResult_t r = ncclAllGather(send, recv, (size_t)send_count, t, reinterpret_cast<ncclComm_t>(comm),
                                         as_stream(stream));
    return r == ncclSuccess ? SKYRL_OK : nccl_fail("ncclAllGather", r);
}

extern "C" int skyrl_comm_broadcast(const void* send, void* recv, int64_t count, int dtype, int32_t root, void* comm,
                                    void* stream) {
    SKYRL_COMM_ARGS("comm_broadcast");
    SKYRL_REQUIRE(count >= 0 && (count == 0 || recv), "comm_broadcast: bad buffers");
    const ncclResult_t r = ncclBroadcast(send, recv, (size_t)count, t, root, reinterpret_cast<ncclComm_t>(comm),
                                         as_stream(stream));
    return r == ncclSuccess ? SKYRL_OK : nccl_fail("ncclBroadcast", r);
}

#undef SKYRL_COMM_ARGS
