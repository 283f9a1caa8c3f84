/*
 * comm.cpp -- the cross-agent collective of the keyframe exchange (include/orbslam_amd.h "Cross-agent collective"):
 * one RCCL all-gather over xGMI of every agent's keyframe slot, issued on a stream the caller chooses.
 *
 * Replaces the reference's LCM publish / subscribe of keyframes between the two agents
 * (ORB_SLAM2.1/Examples/ROS/ORB_SLAM2/src/ros_mono.cc:2399 publishes, ORB_SLAM2/Examples/ROS/ORB_SLAM2/src/
 * ros_mono.cc:602 subscribes). torch.distributed's ProcessGroupNCCL would run the same ncclAllGather on its own
 * internal stream and join it to the caller's with events: one more HIP stream per process beside the bench's graph
 * streams, which share the process's 4 hardware queues. Here the all-gather is enqueued on the caller's
 * stream itself (graph 0's, in order after the keyframe pack), so a rank at N > 1 runs exactly the streams of N = 1.
 *
 * RCCL is bound at run time (dlopen), so liborbamd.so keeps no link dependency on it: inside a process that already
 * loaded torch's librccl.so.1 that copy is reused (RTLD_NOLOAD), else the ROCm one is loaded.
 */
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <mutex>

#include "../../include/orbslam_amd.h"

namespace {

typedef int nccl_result;  // ncclResult_t: 0 = ncclSuccess
typedef void* nccl_comm;  // ncclComm_t
struct nccl_id {
    char internal[ORBX_COMM_ID_BYTES];
};
constexpr int kNcclUint8 = 1;  // ncclDataType_t ncclUint8 (rccl.h)

struct Rccl {
    void* so = nullptr;
    nccl_result (*get_unique_id)(nccl_id*) = nullptr;
    nccl_result (*comm_init_rank)(nccl_comm*, int, nccl_id, int) = nullptr;
    nccl_result (*all_gather)(const void*, void*, size_t, int, nccl_comm, hipStream_t) = nullptr;
    nccl_result (*comm_destroy)(nccl_comm) = nullptr;
    bool ok = false;
};

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        const char* names[] = {"librccl.so.1", "librccl.so"};
        for (const char* n : names)  // torch's copy when this process already holds one
            if ((r.so = dlopen(n, RTLD_NOW | RTLD_NOLOAD))) break;
        if (!r.so)
            for (const char* n : names)
                if ((r.so = dlopen(n, RTLD_NOW | RTLD_LOCAL))) break;
        if (!r.so) return;
        r.get_unique_id = (nccl_result(*)(nccl_id*))dlsym(r.so, "ncclGetUniqueId");
        r.comm_init_rank = (nccl_result(*)(nccl_comm*, int, nccl_id, int))dlsym(r.so, "ncclCommInitRank");
        r.all_gather = (nccl_result(*)(const void*, void*, size_t, int, nccl_comm, hipStream_t))dlsym(r.so, "ncclAllGather");
        r.comm_destroy = (nccl_result(*)(nccl_comm))dlsym(r.so, "ncclCommDestroy");
        r.ok = r.get_unique_id && r.comm_init_rank && r.all_gather && r.comm_destroy;
    });
    return r;
}

}  // namespace

struct orbx_comm {
    nccl_comm comm = nullptr;
    int world = 0, rank = 0, device = 0;
};

extern "C" {

int orbx_comm_unique_id(uint8_t* id) {
    if (!id) return ORBX_EARG;
    const Rccl& r = rccl();
    if (!r.ok) return ORBX_EDEVICE;
    nccl_id u;
    if (r.get_unique_id(&u) != 0) return ORBX_EDEVICE;
    memcpy(id, u.internal, ORBX_COMM_ID_BYTES);
    return 0;
}

int orbx_comm_create(const uint8_t* id, int world, int rank, int device, orbx_comm** out) {
    if (!id || !out || world < 1 || rank < 0 || rank >= world || device < 0) return ORBX_EARG;
    *out = nullptr;
    const Rccl& r = rccl();
    if (!r.ok) return ORBX_EDEVICE;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device >= ndev || hipSetDevice(device) != hipSuccess) {
        (void)hipGetLastError();
        return ORBX_EDEVICE;
    }
    nccl_id u;
    memcpy(u.internal, id, ORBX_COMM_ID_BYTES);
    orbx_comm* c = new orbx_comm();
    c->world = world;
    c->rank = rank;
    c->device = device;
    if (r.comm_init_rank(&c->comm, world, u, rank) != 0) {  // collective: every rank of the world calls it
        delete c;
        return ORBX_EDEVICE;
    }
    *out = c;
    return 0;
}

int orbx_comm_allgather(orbx_comm* c, const void* d_send, void* d_recv, size_t bytes, void* stream) {
    if (!c || (bytes && (!d_send || !d_recv))) return ORBX_EARG;
    if (!bytes) return 0;
    if (hipSetDevice(c->device) != hipSuccess) {
        (void)hipGetLastError();
        return ORBX_EDEVICE;
    }
    if (rccl().all_gather(d_send, d_recv, bytes, kNcclUint8, c->comm, (hipStream_t)stream) != 0) return ORBX_EDEVICE;
    return 0;
}

void orbx_comm_destroy(orbx_comm* c) {
    if (!c) return;
    if (c->comm) (void)rccl().comm_destroy(c->comm);
    delete c;
}

}  // extern "C"
