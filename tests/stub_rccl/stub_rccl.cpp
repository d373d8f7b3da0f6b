// stub_rccl.cpp -- TEST INFRASTRUCTURE: the RCCL entry points the engine's in-process key replication
// calls (engine.hip replicate_arena: ncclCommInitAll, ncclGroupStart, ncclBroadcast per device,
// ncclGroupEnd, ncclCommDestroy, ncclGetErrorString), implemented with HIP device copies so that the
// group / sync / destroy sequence runs on a one-GPU box, where TFHE_LOGICAL_DEVICES puts every logical
// device on the same GPU (a real communicator cannot hold a device twice).  Selected with
// TFHE_RCCL_LIB=<this library> at tfhe_setup (tests/test_gpu_rccl_stub.py).
//
// Semantics kept from RCCL: inside a group, broadcasts are recorded and issued at ncclGroupEnd; a
// non-root rank's send buffer is ignored -- it receives the root's buffer, ordered after the root's
// stream by an event; the calls return before the copies complete (the caller synchronises its streams).
// STUB_RCCL_FAIL=init makes ncclCommInitAll fail (the engine must fall back to peer copies);
// STUB_RCCL_FAIL=short delivers only the first half of each broadcast (the engine's replica checksum
// must fail the setup).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

namespace {
struct Shared {
    int nranks = 0;
};
struct Op {
    const void* send;
    void* recv;
    size_t bytes;
    int root;
    int rank;
    int device;
    hipStream_t stream;
};
std::mutex g_mu;
std::vector<Op> g_pending;
int g_depth = 0;
std::atomic<int> g_broadcasts{0}, g_groups{0}, g_comms{0};

size_t type_bytes(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        default: return 8;
    }
}

ncclResult_t flush() {  // issue the recorded broadcasts (caller holds g_mu)
    for (const Op& root : g_pending) {
        if (root.rank != root.root) continue;
        hipEvent_t ready;
        if (hipSetDevice(root.device) != hipSuccess ||
            hipEventCreateWithFlags(&ready, hipEventDisableTiming) != hipSuccess ||
            hipEventRecord(ready, root.stream) != hipSuccess)
            return ncclUnhandledCudaError;
        for (const Op& op : g_pending) {
            if (op.rank == op.root) {
                if (op.recv != op.send &&
                    hipMemcpyAsync(op.recv, op.send, op.bytes, hipMemcpyDeviceToDevice, op.stream) != hipSuccess)
                    return ncclUnhandledCudaError;
                continue;
            }
            const char* f = std::getenv("STUB_RCCL_FAIL");
            const size_t bytes = f && std::strcmp(f, "short") == 0 ? op.bytes / 2 : op.bytes;
            if (hipSetDevice(op.device) != hipSuccess || hipStreamWaitEvent(op.stream, ready, 0) != hipSuccess ||
                hipMemcpyAsync(op.recv, root.send, bytes, hipMemcpyDeviceToDevice, op.stream) != hipSuccess)
                return ncclUnhandledCudaError;
            ++g_broadcasts;
        }
        (void)hipEventDestroy(ready);
    }
    g_pending.clear();
    return ncclSuccess;
}
}  // namespace

struct ncclComm {
    Shared* sh;
    int rank;
    int device;
};

extern "C" {

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
    const char* f = std::getenv("STUB_RCCL_FAIL");
    if (f && std::strcmp(f, "init") == 0) return ncclSystemError;
    auto* sh = new Shared{ndev};
    for (int i = 0; i < ndev; ++i) comms[i] = new ncclComm{sh, i, devlist ? devlist[i] : i};
    g_comms += ndev;
    return ncclSuccess;
}

ncclResult_t ncclGetVersion(int* version) {
    if (!version) return ncclInvalidArgument;
    *version = 0;  // the stub: no RCCL version
    return ncclSuccess;
}

ncclResult_t ncclGroupStart() {
    std::lock_guard<std::mutex> l(g_mu);
    ++g_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    std::lock_guard<std::mutex> l(g_mu);
    if (g_depth == 0) return ncclInvalidUsage;
    ++g_groups;
    return --g_depth == 0 ? flush() : ncclSuccess;
}

ncclResult_t ncclBroadcast(const void* sendbuff, void* recvbuff, size_t count, ncclDataType_t datatype, int root,
                           ncclComm_t comm, hipStream_t stream) {
    if (!comm || root < 0 || root >= comm->sh->nranks) return ncclInvalidArgument;
    std::lock_guard<std::mutex> l(g_mu);
    g_pending.push_back(Op{sendbuff, recvbuff, count * type_bytes(datatype), root, comm->rank, comm->device, stream});
    return g_depth == 0 ? flush() : ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    if (!comm) return ncclInvalidArgument;
    if (comm->rank == 0) delete comm->sh;
    delete comm;
    return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) { return r == ncclSuccess ? "no error" : "stub rccl error"; }

// test hooks: how many non-root receives were issued, how many groups closed, communicators made
int stub_rccl_broadcasts() { return g_broadcasts.load(); }
int stub_rccl_groups() { return g_groups.load(); }
int stub_rccl_comms() { return g_comms.load(); }

}  // extern "C"
