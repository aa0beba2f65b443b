#pragma once
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>

#include <memory>
#include <string>
#include <vector>

namespace dlmpi_ext {

// Native RCCL communicator (one per process / GPU) with a dedicated comm stream.
class RcclComm {
 public:
  static pybind11::bytes unique_id();
  // max_ctas > 0: this communicator's channel (workgroup) cap, through ncclCommInitRankConfig
  // (maxCTAs) -- per communicator, unlike NCCL_MAX_NCHANNELS, which RCCL reads once per process
  RcclComm(const std::string& uid, int rank, int size, int device, int max_ctas = 0);
  ~RcclComm();
  int rank() const;
  int size() const;
  int max_ctas() const;
  int64_t stream_handle() const;
  void fence_in();
  void fence_out();
  void allreduce_async(at::Tensor t, const std::string& op);
  void allreduce(at::Tensor t, const std::string& op, bool async_op);
  void broadcast(at::Tensor t, int root, bool async_op);
  void allgather(at::Tensor out, const at::Tensor& in, bool async_op);
  void reduce_scatter(at::Tensor out, const at::Tensor& in, const std::string& op, bool async_op);
  void alltoall(at::Tensor out, const at::Tensor& in, bool async_op);
  void send(const at::Tensor& t, int peer);
  void recv(at::Tensor t, int peer);
  void wait();
  void synchronize();
  void barrier();
  void destroy();
  // After a failed hipGraph capture that had forked the comm stream: if the stream is still in
  // capture mode (HIP leaves an invalidated capture open), switch to a fresh stream.  Returns true
  // if the stream was replaced.
  bool reset_stream_if_capturing();

 private:
  void record(const at::Tensor& t);
  struct Impl;
  std::unique_ptr<Impl> impl_;
};

// What the reducer needs from a communication backend.  Implemented natively over RCCL
// (RcclBucketComm) and, for CPU / gloo testing, by a Python subclass (PyCommBase trampoline).
class CommBase {
 public:
  virtual ~CommBase() = default;
  virtual void begin_step() {}     // a synchronised step starts (Reducer::prepare_for_backward, DDP forward)
  virtual void begin_bucket() {}
  virtual void allreduce_bucket(at::Tensor t, bool average) = 0;
  virtual void end_backward() {}
};

class PyCommBase : public CommBase {
 public:
  using CommBase::CommBase;
  void begin_step() override { PYBIND11_OVERRIDE(void, CommBase, begin_step, ); }
  void begin_bucket() override { PYBIND11_OVERRIDE(void, CommBase, begin_bucket, ); }
  void allreduce_bucket(at::Tensor t, bool average) override {
    PYBIND11_OVERRIDE_PURE(void, CommBase, allreduce_bucket, t, average);
  }
  void end_backward() override { PYBIND11_OVERRIDE(void, CommBase, end_backward, ); }
};

class RcclBucketComm : public CommBase {
 public:
  explicit RcclBucketComm(std::shared_ptr<RcclComm> c) : comm_(std::move(c)) {}
  ~RcclBucketComm() override;
  void begin_step() override;
  void begin_bucket() override;
  void allreduce_bucket(at::Tensor t, bool average) override;
  void end_backward() override;
  // Per-bucket timing (off by default; never inside a hipGraph capture): timing events at the step's
  // start (begin_step: the DDP forward, compute stream), around every bucket all-reduce (comm stream)
  // and at the end of the backward's compute (compute stream, before it waits for the comm stream).
  void set_timing(bool on) { timing_ = on; }
  // The last timed step (synchronises its events): per bucket {bytes, start_ms, dur_ms} with start_ms
  // relative to the step's start, and compute_end_ms.
  pybind11::dict timings();

 private:
  hipEvent_t tev();
  std::shared_ptr<RcclComm> comm_;
  bool timing_ = false;
  std::vector<hipEvent_t> pool_;
  size_t used_ = 0;
  hipEvent_t ref_ = nullptr, cend_ = nullptr;
  struct Rec {
    int64_t bytes;
    hipEvent_t a, b;
  };
  std::vector<Rec> recs_;
};

// One-GPU rehearsal of an N-rank all-reduce's cost to the compute streams (comm.cpp): the real
// (world-size-1) RCCL all-reduce, followed on the comm stream by a load kernel that occupies
// `channels` workgroups with `lds_bytes` of LDS each, moves the ring all-reduce's per-rank traffic
// 2 (W-1)/W * bytes, and holds the CUs for the modeled collective time
// 2 (W-1)/W * bytes / min(gbps_max, channels * gbps_per_channel) + latency_us.
class RehearsalBucketComm : public CommBase {
 public:
  RehearsalBucketComm(std::shared_ptr<RcclComm> c, int world, int channels, int lds_bytes, double gbps_per_channel,
                      double gbps_max, double latency_us);
  void begin_bucket() override;
  void allreduce_bucket(at::Tensor t, bool average) override;
  void end_backward() override;
  double modeled_us_total() const { return modeled_us_; }   // sum over buckets since construction
  int64_t buckets() const { return nbuckets_; }

 private:
  std::shared_ptr<RcclComm> comm_;
  int world_, channels_, lds_;
  double gbps_ch_, gbps_max_, lat_us_;
  at::Tensor scratch_;
  double modeled_us_ = 0.0;
  int64_t nbuckets_ = 0;
};

// Gradient-bucket reducer (see comm.cpp).
class Reducer {
 public:
  Reducer(std::vector<at::Tensor> buckets, std::vector<int64_t> param_bucket, std::shared_ptr<CommBase> comm,
          bool average);
  void prepare_for_backward();
  void mark_ready(int64_t param_idx);
  void finalize();
  int64_t num_buckets() const { return (int64_t)buckets_.size(); }
  int64_t launched() const { return launched_; }

 private:
  void launch_ready();
  std::vector<at::Tensor> buckets_;
  std::vector<int64_t> param_bucket_;
  std::shared_ptr<CommBase> comm_;
  bool average_;
  std::vector<int64_t> expected_, pending_;
  std::vector<char> seen_;
  int64_t next_ = 0, launched_ = 0;
};

void register_comm(pybind11::module& m);

}  // namespace dlmpi_ext
