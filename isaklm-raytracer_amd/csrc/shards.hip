// shards.hip — the multi-GPU closing step of SURVEY §8e as C-ABI calls:
// one RCCL reduce(sum) of every shard's G_Buffer accumulators (fb, sq,
// count) into the root over xGMI.  Replaces nothing in the reference (it is
// single-GPU); it is the `rt_reduce_shards` entry point §8b asks for, so a C++
// caller can shard without torch.  bench.py drives the same reduce through
// torch.distributed (its RCCL backend); both are one ncclReduce per array.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include "../../include/isaklm_rt.h"

void rt_set_error(const char *fmt, ...);

struct RtComm {
    ncclComm_t comm;
    int nranks, rank;
};

static_assert(sizeof(ncclUniqueId) == RT_COMM_ID_BYTES, "RT_COMM_ID_BYTES");

#define NCCLCHK(x)                                                                  \
    do {                                                                            \
        ncclResult_t r_ = (x);                                                      \
        if (r_ != ncclSuccess) {                                                    \
            rt_set_error("%s: %s", #x, ncclGetErrorString(r_));                     \
            return RT_E_HIP;                                                        \
        }                                                                           \
    } while (0)

extern "C" {

int rt_comm_unique_id(void *id_out)
{
    if (!id_out) { rt_set_error("rt_comm_unique_id: null"); return RT_E_INVALID; }
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    memcpy(id_out, &id, sizeof id);
    return RT_OK;
}

int rt_comm_create(int nranks, int rank, const void *id, rt_comm_t *out)
{
    if (!id || !out || nranks < 1 || rank < 0 || rank >= nranks) {
        rt_set_error("rt_comm_create: bad arguments");
        return RT_E_INVALID;
    }
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    RtComm *c = new RtComm();
    c->nranks = nranks;
    c->rank = rank;
    ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        rt_set_error("ncclCommInitRank: %s", ncclGetErrorString(r));
        delete c;
        return RT_E_HIP;
    }
    *out = c;
    return RT_OK;
}

int rt_comm_destroy(rt_comm_t c)
{
    if (!c) return RT_OK;
    ncclResult_t r = ncclCommDestroy(c->comm);
    delete c;
    if (r != ncclSuccess) {
        rt_set_error("ncclCommDestroy: %s", ncclGetErrorString(r));
        return RT_E_HIP;
    }
    return RT_OK;
}

int rt_reduce_shards(rt_comm_t c, G_Buffer g, int width, int height, int root, void *stream)
{
    if (!c || !g.frame_buffer || !g.squared_luminance || !g.sample_count || width <= 0 || height <= 0 ||
        root < 0 || root >= c->nranks) {
        rt_set_error("rt_reduce_shards: bad arguments");
        return RT_E_INVALID;
    }
    const size_t n = (size_t)width * height;
    hipStream_t s = (hipStream_t)stream;
    if (rt_join(stream) != RT_OK) return RT_E_HIP; // chained renders' deep-path tails first
    NCCLCHK(ncclGroupStart());
    NCCLCHK(ncclReduce(g.frame_buffer, g.frame_buffer, 3 * n, ncclFloat32, ncclSum, root, c->comm, s));
    NCCLCHK(ncclReduce(g.squared_luminance, g.squared_luminance, n, ncclFloat32, ncclSum, root, c->comm, s));
    NCCLCHK(ncclReduce(g.sample_count, g.sample_count, n, ncclInt32, ncclSum, root, c->comm, s));
    NCCLCHK(ncclGroupEnd());
    if (!stream && hipStreamSynchronize(nullptr) != hipSuccess) {
        rt_set_error("rt_reduce_shards: %s", hipGetErrorString(hipGetLastError()));
        return RT_E_HIP;
    }
    return RT_OK;
}

} // extern "C"
