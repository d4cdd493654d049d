// Native RCCL communicator: the MI355X data plane that replaces the
// reference's libipc TCP sockets + ipc.Tree b-ary tree.
//
//  reference                                    here
//  -------------------------------------------  -------------------------------------------
//  tree.allReduce(value, add)  (AllReduceSGD:12) all_reduce -> ncclAllReduce(sum) on a flat
//                                                 bucket, issued on the caller's HIP stream
//  tree.scatter(value)         (AllReduceSGD:52) broadcast -> ncclBroadcast(root)
//  client:send / client:recv   (AsyncEA:87-130)  send / recv -> ncclSend / ncclRecv (grouped)
//  ipc.server/ipc.client rendezvous             ncclUniqueId exchanged through the c10d TCPStore
//
// The communicator never synchronises the host: every call is enqueued on a
// stream handle supplied by Python (a torch stream), so calls are legal inside
// hipGraph capture and can be overlapped with compute on a side stream.
#pragma once
#include <rccl/rccl.h>

#include <cstring>
#include <string>
#include <vector>

#include "dl_common.h"

#define DL_NCCL_CHECK(expr)                                                                                      \
  do {                                                                                                           \
    ncclResult_t _r = (expr);                                                                                    \
    if (_r != ncclSuccess) {                                                                                     \
      throw std::runtime_error(std::string("RCCL error: ") + ncclGetErrorString(_r) + " at " + __FILE__ + ":" + \
                               std::to_string(__LINE__));                                                        \
    }                                                                                                            \
  } while (0)

namespace dl {

// dtype codes shared with python (torch_distlearn_amd/parallel/comm.py)
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2, kI64 = 3, kI32 = 4, kU8 = 5, kF64 = 6 };
enum ROp : int { kSum = 0, kProd = 1, kMax = 2, kMin = 3, kAvg = 4 };

inline ncclDataType_t to_nccl(int dt) {
  switch (dt) {
    case kF32: return ncclFloat32;
    case kBF16: return ncclBfloat16;
    case kF16: return ncclFloat16;
    case kI64: return ncclInt64;
    case kI32: return ncclInt32;
    case kU8: return ncclUint8;
    case kF64: return ncclFloat64;
  }
  throw std::runtime_error("unsupported dtype code " + std::to_string(dt));
}

inline ncclRedOp_t to_nccl_op(int op) {
  switch (op) {
    case kSum: return ncclSum;
    case kProd: return ncclProd;
    case kMax: return ncclMax;
    case kMin: return ncclMin;
    case kAvg: return ncclAvg;
  }
  throw std::runtime_error("unsupported reduction op " + std::to_string(op));
}

inline std::string rccl_unique_id() {
  ncclUniqueId id;
  DL_NCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

inline int rccl_version() {
  int v = 0;
  DL_NCCL_CHECK(ncclGetVersion(&v));
  return v;
}

class RcclCommunicator {
 public:
  RcclCommunicator(const std::string& uid, int rank, int world, int device) : rank_(rank), world_(world), dev_(device) {
    if ((int)uid.size() != (int)sizeof(ncclUniqueId)) throw std::runtime_error("bad ncclUniqueId size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    DL_HIP_CHECK(hipSetDevice(device));
    DL_NCCL_CHECK(ncclCommInitRank(&comm_, world, id, rank));
  }
  ~RcclCommunicator() { destroy(); }

  void destroy() {
    if (comm_) {
      ncclCommDestroy(comm_);
      comm_ = nullptr;
    }
  }
  void abort() {
    if (comm_) {
      ncclCommAbort(comm_);
      comm_ = nullptr;
    }
  }

  int rank() const { return rank_; }
  int world() const { return world_; }
  int device() const { return dev_; }

  void all_reduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, uintptr_t stream) {
    live();
    DL_NCCL_CHECK(ncclAllReduce((const void*)send, (void*)recv, (size_t)count, to_nccl(dtype), to_nccl_op(op), comm_,
                                as_stream(stream)));
  }
  void broadcast(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int root, uintptr_t stream) {
    live();
    DL_NCCL_CHECK(
        ncclBroadcast((const void*)send, (void*)recv, (size_t)count, to_nccl(dtype), root, comm_, as_stream(stream)));
  }
  void reduce(uintptr_t send, uintptr_t recv, int64_t count, int dtype, int op, int root, uintptr_t stream) {
    live();
    DL_NCCL_CHECK(ncclReduce((const void*)send, (void*)recv, (size_t)count, to_nccl(dtype), to_nccl_op(op), root,
                             comm_, as_stream(stream)));
  }
  // recvcount elements per rank
  void reduce_scatter(uintptr_t send, uintptr_t recv, int64_t recvcount, int dtype, int op, uintptr_t stream) {
    live();
    DL_NCCL_CHECK(ncclReduceScatter((const void*)send, (void*)recv, (size_t)recvcount, to_nccl(dtype),
                                    to_nccl_op(op), comm_, as_stream(stream)));
  }
  void all_gather(uintptr_t send, uintptr_t recv, int64_t sendcount, int dtype, uintptr_t stream) {
    live();
    DL_NCCL_CHECK(
        ncclAllGather((const void*)send, (void*)recv, (size_t)sendcount, to_nccl(dtype), comm_, as_stream(stream)));
  }
  void send(uintptr_t buf, int64_t count, int dtype, int peer, uintptr_t stream) {
    live();
    DL_NCCL_CHECK(ncclSend((const void*)buf, (size_t)count, to_nccl(dtype), peer, comm_, as_stream(stream)));
  }
  void recv(uintptr_t buf, int64_t count, int dtype, int peer, uintptr_t stream) {
    live();
    DL_NCCL_CHECK(ncclRecv((void*)buf, (size_t)count, to_nccl(dtype), peer, comm_, as_stream(stream)));
  }
  void group_start() { DL_NCCL_CHECK(ncclGroupStart()); }
  void group_end() { DL_NCCL_CHECK(ncclGroupEnd()); }

  // Non-blocking health check (failure detection). Returns the
  // RCCL async error string or "" when healthy.
  std::string async_error() {
    if (!comm_) return "communicator destroyed";
    ncclResult_t r;
    DL_NCCL_CHECK(ncclCommGetAsyncError(comm_, &r));
    if (r == ncclSuccess || r == ncclInProgress) return "";
    return ncclGetErrorString(r);
  }

 private:
  void live() const {
    if (!comm_) throw std::runtime_error("RCCL communicator used after destroy/abort");
  }
  ncclComm_t comm_ = nullptr;
  int rank_, world_, dev_;
};

}  // namespace dl
