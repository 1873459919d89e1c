// ricepp_facade.cpp -- C++ host facade (include/ricepp_amd.hpp) over the C ABI.
//
// The DwarFS plugin semantics follow src/compression/ricepp.cpp (file:line
// cited at each method).  Encode / decode calls go through a per-(device,
// config) combining queue: concurrent calls are coalesced into one
// rpp_encode_batch_ws / rpp_decode_batch_ws launch on a pooled device context
// (stream + grow-only device arena + grow-only pinned staging), so the
// worker_group threads of the DwarFS writer (src/writer/filesystem_writer.cpp:
// 255-287) and block cache (src/reader/internal/block_cache.cpp:628-706) feed
// the GPU in batches without any per-call stream creation or allocation.
#include "ricepp_amd.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <charconv>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <string>
#include <tuple>

namespace ricepp_amd {

namespace {

void hip_check(hipError_t e, char const* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("ricepp_amd: ") + what + ": " + hipGetErrorString(e));
}

rpp_config to_rpp(codec_config const& c) {
  rpp_config r{};
  r.block_size = c.block_size > 0xFFFFFFFFu ? 0xFFFFFFFFu : static_cast<uint32_t>(c.block_size);
  r.component_stream_count =
      c.component_stream_count > 0xFFFFFFFFu ? 0xFFFFFFFFu : static_cast<uint32_t>(c.component_stream_count);
  r.big_endian = c.byteorder == std::endian::big ? 1u : 0u;
  r.unused_lsb_count = c.unused_lsb_count;
  return r;
}

[[noreturn]] void throw_status(int st) {
  switch (st) {
    case RPP_UNSUPPORTED_CONFIG: throw std::runtime_error("Unsupported configuration");
    case RPP_TRUNCATED_INPUT: throw std::out_of_range("bitstream_reader::read_packet");
    case RPP_INVALID_ARGUMENT: throw std::invalid_argument("ricepp_amd: invalid argument");
    case RPP_OUTPUT_TOO_SMALL: throw std::length_error("ricepp_amd: output buffer too small");
    case RPP_INTERNAL_ERROR: throw std::runtime_error("ricepp_amd: internal error (device consistency bound)");
    default: throw std::runtime_error("ricepp_amd: HIP error");
  }
}

size_t align16(size_t v) { return (v + 15) & ~size_t{15}; }

std::atomic<uint64_t> g_enc_launches{0}, g_enc_blocks{0}, g_dec_launches{0}, g_dec_blocks{0}, g_ctx_created{0};
std::atomic<uint32_t> g_ctx_faults{0};  // inject_context_failures
std::atomic<uint64_t> g_stage_ns{0}, g_device_ns{0}, g_finish_ns{0};
inline uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int current_device() {
  int d = 0;
  hip_check(hipGetDevice(&d), "hipGetDevice");
  return d;
}

// Makes `dev` current for the calling thread for the guard's lifetime.
class device_guard {
 public:
  explicit device_guard(int dev) : dev_{dev} {
    hip_check(hipGetDevice(&prev_), "hipGetDevice");
    if (prev_ != dev_) hip_check(hipSetDevice(dev_), "hipSetDevice");
  }
  ~device_guard() {
    if (prev_ != dev_) (void)hipSetDevice(prev_);
  }
  device_guard(device_guard const&) = delete;
  device_guard& operator=(device_guard const&) = delete;

 private:
  int dev_;
  int prev_ = 0;
};

// A private stream plus device and pinned host buffers, bound to one device.
// Device buffers come from the stream-ordered allocator (hipMallocAsync /
// hipFreeAsync on the context's stream), so growing one never synchronises the
// device.  Pinned buffers are mapped into the device's address space (the
// encoder packs its output straight into them) and grow geometrically; a
// context going back to the pool drops pinned buffers above kPinnedKeep, so a
// burst of huge batches does not keep GiBs of host memory pinned.
constexpr size_t kPinnedKeep = size_t{64} << 20;

class device_ctx {
 public:
  explicit device_ctx(int dev) : dev_{dev} {
    for (uint32_t n = g_ctx_faults.load(); n;)
      if (g_ctx_faults.compare_exchange_weak(n, n - 1)) throw std::runtime_error("hipStreamCreate: injected failure");
    device_guard g{dev_};
    hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    g_ctx_created.fetch_add(1, std::memory_order_relaxed);
  }
  device_ctx(device_ctx const&) = delete;
  device_ctx& operator=(device_ctx const&) = delete;

  int device() const { return dev_; }
  hipStream_t stream() const { return stream_; }
  uint8_t* dev(size_t bytes) { return grow_dev(dbuf_, dcap_, bytes); }
  uint8_t* workspace(size_t bytes) { return grow_dev(wbuf_, wcap_, bytes); }
  uint8_t* pin_in(size_t bytes) { return grow_pinned(hin_, hin_cap_, bytes); }
  uint8_t* pin_out(size_t bytes) { return grow_pinned(hout_, hout_cap_, bytes); }
  // the device-side address of a pinned buffer
  uint8_t* device_view(uint8_t* pinned) {
    void* d = nullptr;
    hip_check(hipHostGetDevicePointer(&d, pinned, 0), "hipHostGetDevicePointer");
    return static_cast<uint8_t*>(d);
  }
  void sync() { hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize"); }
  // on release (the stream is idle: every batch ends with a sync)
  void trim() {
    for (auto* q : {&hin_, &hout_}) {
      size_t& cap = q == &hin_ ? hin_cap_ : hout_cap_;
      if (cap > kPinnedKeep) {
        (void)hipHostFree(*q);
        *q = nullptr;
        cap = 0;
      }
    }
  }

 private:
  uint8_t* grow_dev(uint8_t*& p, size_t& cap, size_t bytes) {
    if (bytes <= cap && p) return p;
    size_t n = cap ? cap : size_t{1} << 20;
    while (n < bytes) n *= 2;
    if (p) (void)hipFreeAsync(p, stream_);  // (stream-ordered: after the work that used it)
    p = nullptr;
    cap = 0;
    void* q = nullptr;
    hip_check(hipMallocAsync(&q, n, stream_), "hipMallocAsync");
    p = static_cast<uint8_t*>(q);
    cap = n;
    return p;
  }
  // (pinned buffers only grow between batches: the stream is idle then)
  static uint8_t* grow_pinned(uint8_t*& p, size_t& cap, size_t bytes) {
    if (bytes <= cap && p) return p;
    size_t n = cap ? cap : size_t{1} << 20;
    while (n < bytes) n *= 2;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    void* q = nullptr;
    hip_check(hipHostMalloc(&q, n, hipHostMallocMapped), "hipHostMalloc");
    p = static_cast<uint8_t*>(q);
    cap = n;
    return p;
  }

  int dev_;
  hipStream_t stream_ = nullptr;
  uint8_t* dbuf_ = nullptr;
  size_t dcap_ = 0;
  uint8_t* wbuf_ = nullptr;
  size_t wcap_ = 0;
  uint8_t* hin_ = nullptr;
  size_t hin_cap_ = 0;
  uint8_t* hout_ = nullptr;
  size_t hout_cap_ = 0;
};

// Per-device free lists of contexts (intentionally leaked at exit: no HIP
// calls from static destructors).
class ctx_pool {
 public:
  static ctx_pool& get() {
    static ctx_pool* p = new ctx_pool;
    return *p;
  }
  device_ctx* acquire(int dev) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto& v = free_[dev];
      if (!v.empty()) {
        device_ctx* c = v.back();
        v.pop_back();
        return c;
      }
    }
    return new device_ctx(dev);
  }
  void release(device_ctx* c) {
    c->trim();
    std::lock_guard<std::mutex> lk(mu_);
    free_[c->device()].push_back(c);
  }

 private:
  std::mutex mu_;
  std::map<int, std::vector<device_ctx*>> free_;
};

class ctx_lease {
 public:
  explicit ctx_lease(int dev) : c_{ctx_pool::get().acquire(dev)} {}
  ~ctx_lease() { ctx_pool::get().release(c_); }
  ctx_lease(ctx_lease const&) = delete;
  ctx_lease& operator=(ctx_lease const&) = delete;
  device_ctx& operator*() const { return *c_; }
  device_ctx* operator->() const { return c_; }

 private:
  device_ctx* c_;
};

// ---- combining batch queue ----
//
// A request moves QUEUED -> TAKEN (in a batch) -> ASSIGNED (its pinned input
// slot is known: the caller copies its input in) -> STAGED -> RESULT (its
// pinned output slot is filled: the caller copies its output out) -> DONE.
// The first waiting caller that finds a free launch slot takes everything
// queued (up to the batch caps) and drives the launch; every caller does its
// own host copies, in parallel.  The leader only touches a request through
// the batch's counters once the request may have returned.  Up to kMaxActive
// batches of one queue are in flight at once, each on its own pooled context
// (stream), and each costs one host synchronisation.
enum req_state { QUEUED, TAKEN, ASSIGNED, STAGED, RESULT, DONE };

struct batch_counts {
  size_t to_stage = 0;   // requests not yet STAGED
  size_t to_finish = 0;  // requests not yet DONE
  std::condition_variable cv;  // the leader waits here
};

struct request {
  // encode: in = samples, out = caller's output; decode: in = stream bytes,
  // out = sample bytes
  uint8_t const* in;
  size_t in_bytes;
  uint8_t* out;
  size_t out_cap;  // encode: output span size; decode: exact sample bytes
  uint64_t n_samples;
  // set by the leader
  uint8_t* pin_in = nullptr;
  uint8_t const* pin_out = nullptr;
  size_t result_bytes = 0;
  int status = RPP_OK;
  std::string error;  // HIP failure text
  req_state state = QUEUED;
  batch_counts* counts = nullptr;
  std::condition_variable cv;  // its caller waits here (woken individually: no notify_all storms)
};

constexpr size_t kMaxBatchBlocks = 8192;
constexpr size_t kMaxBatchBytes = size_t{512} << 20;  // input + output bytes per launch
// launches in flight per queue: HIP maps a process's streams onto
// GPU_MAX_HW_QUEUES hardware queues (4 by default), so more concurrent launches
// only queue behind each other on the device (measured: 16 in flight took the
// 64-thread decode from 4.5 to 1.4 GiB/s); fewer, bigger batches win
constexpr int kMaxActive = 4;

class batch_queue {
 public:
  batch_queue(int dev, rpp_config cfg, bool encode) : dev_{dev}, cfg_{cfg}, encode_{encode} {}

  void run(request& r) {
    std::unique_lock<std::mutex> lk(mu_);
    pending_.push_back(&r);
    for (;;) {
      switch (r.state) {
        case DONE: return;
        case ASSIGNED: copy_in(lk, r); continue;
        case RESULT: copy_out(lk, r); return;
        case QUEUED:
          if (active_ < kMaxActive) {
            lead(lk, r);
            continue;
          }
          break;
        default: break;
      }
      r.cv.wait(lk);
    }
  }

 private:
  // bytes a request moves through a launch (input, and output capacity)
  size_t footprint(request const* q) const {
    return q->in_bytes + (encode_ ? rpp_worst_case_bytes(&cfg_, q->n_samples) : q->out_cap);
  }
  void copy_in(std::unique_lock<std::mutex>& lk, request& r) {
    lk.unlock();
    if (r.in_bytes) std::memcpy(r.pin_in, r.in, r.in_bytes);
    lk.lock();
    r.state = STAGED;
    if (--r.counts->to_stage == 0) r.counts->cv.notify_one();
  }
  void copy_out(std::unique_lock<std::mutex>& lk, request& r) {
    lk.unlock();
    if (r.status == RPP_OK && r.result_bytes) std::memcpy(r.out, r.pin_out, r.result_bytes);
    lk.lock();
    r.state = DONE;
    batch_counts* c = r.counts;  // (r may be gone once DONE is seen)
    if (--c->to_finish == 0) c->cv.notify_one();
  }

  // Takes a batch from the queue and drives it (lk held on entry and exit).
  // `self` is the leader's own request, which may or may not be in the batch.
  // Every exit path publishes a result to every request of the batch, waits
  // until all of them are DONE, and gives the launch slot back.
  void lead(std::unique_lock<std::mutex>& lk, request& self) {
    std::vector<request*> b;
    size_t bytes = 0;
    while (!pending_.empty() && b.size() < kMaxBatchBlocks &&
           (b.empty() || bytes + footprint(pending_.front()) <= kMaxBatchBytes)) {
      request* q = pending_.front();
      pending_.pop_front();
      bytes += footprint(q);
      q->state = TAKEN;
      b.push_back(q);
    }
    batch_counts counts;
    counts.to_stage = counts.to_finish = b.size();
    for (request* q : b) q->counts = &counts;
    ++active_;
    // another caller may lead the next batch meanwhile
    if (!pending_.empty() && active_ < kMaxActive) pending_.front()->cv.notify_one();
    lk.unlock();
    try {
      ctx_lease ctx{dev_};  // (may throw: no request has a slot yet)
      device_guard g{dev_};
      if (encode_) launch_encode(lk, b, self, *ctx);
      else launch_decode(lk, b, self, *ctx);
      const uint64_t tf = now_ns();
      lk.lock();
      // the leader copies its own result out, then waits for the others
      // before the pinned buffers go back to the pool (with the lease)
      if (self.state == RESULT && self.counts == &counts) copy_out(lk, self);
      counts.cv.wait(lk, [&] { return counts.to_finish == 0; });
      lk.unlock();
      g_finish_ns.fetch_add(now_ns() - tf, std::memory_order_relaxed);
    } catch (std::exception const& e) {
      // thrown before stage_in handed out slots or after every request was
      // STAGED (launch_* only throws outside stage_in): no caller is copying
      lk.lock();
      for (request* q : b)
        if (q->state == TAKEN) {
          q->state = STAGED;
          --counts.to_stage;
        }
      for (request* q : b) {
        if (q->state == RESULT || q->state == DONE) continue;
        q->status = RPP_HIP_ERROR;
        q->error = e.what();
        q->result_bytes = 0;
        q->state = RESULT;
        if (q != &self) q->cv.notify_one();
      }
      if (self.state == RESULT && self.counts == &counts) copy_out(lk, self);
      counts.cv.wait(lk, [&] { return counts.to_finish == 0; });
      lk.unlock();
    }
    lk.lock();
    --active_;
    if (!pending_.empty()) pending_.front()->cv.notify_one();  // the next leader
  }

  // Hands out the pinned input slots and waits until every caller copied in
  // (lk not held on entry or exit).
  void stage_in(std::unique_lock<std::mutex>& lk, std::vector<request*> const& b, request& self, uint8_t* pin,
                std::vector<size_t> const& off) {
    lk.lock();
    for (size_t i = 0; i < b.size(); ++i) {
      b[i]->pin_in = pin + off[i];
      b[i]->state = ASSIGNED;
      if (b[i] != &self) b[i]->cv.notify_one();
    }
    batch_counts* c = b.front()->counts;
    if (self.state == ASSIGNED && self.counts == c) copy_in(lk, self);
    c->cv.wait(lk, [&] { return c->to_stage == 0; });
    lk.unlock();
  }

  // Publishes the results (lk not held on entry or exit).
  void publish(std::unique_lock<std::mutex>& lk, std::vector<request*> const& b, request& self) {
    lk.lock();
    for (request* q : b) {
      q->state = RESULT;
      if (q != &self) q->cv.notify_one();
    }
    lk.unlock();
  }

  // One synchronisation per batch: the packed encoded bytes go straight from
  // the pack kernel into mapped pinned memory, the sizes and statuses follow
  // in one small copy.
  void launch_encode(std::unique_lock<std::mutex>& lk, std::vector<request*> const& b, request& self,
                     device_ctx& ctx) {
    const size_t nb = b.size();
    std::vector<size_t> in_off(nb), out_off(nb);
    size_t in_total = 0, out_total = 0;
    uint64_t total_samples = 0, max_samples = 0;
    for (size_t i = 0; i < nb; ++i) {
      in_off[i] = in_total;
      in_total += align16(b[i]->in_bytes);
      out_off[i] = out_total;
      out_total += align16(rpp_worst_case_bytes(&cfg_, b[i]->n_samples)) + 16;
      total_samples += b[i]->n_samples;
      max_samples = std::max<uint64_t>(max_samples, b[i]->n_samples);
    }
    // device: [in][u64 in_off | n | out_off | out_bytes | dst_off | total][i32 status][out slots]
    // pinned in: [in][u64 in_off | n | out_off]   (one H2D copy)
    // pinned out: [packed bytes][u64 out_bytes | dst_off | total][i32 status]
    const size_t arr = (6 * nb + 1) * 8 + align16(nb * 4);
    uint8_t* d = ctx.dev(in_total + arr + out_total + 64);
    uint8_t* pin = ctx.pin_in(in_total + 3 * nb * 8 + 64);
    uint8_t* pout = ctx.pin_out(out_total + arr + 64);
    auto* h64 = reinterpret_cast<uint64_t*>(pin + in_total);
    for (size_t i = 0; i < nb; ++i) {
      h64[i] = in_off[i] / 2;
      h64[nb + i] = b[i]->n_samples;
      h64[2 * nb + i] = out_off[i];
    }
    const uint64_t ws_bytes = rpp_encode_workspace_bytes(&cfg_, total_samples, max_samples, static_cast<uint32_t>(nb));
    uint8_t* ws = ws_bytes ? ctx.workspace(ws_bytes) : nullptr;
    uint8_t* pout_dev = ctx.device_view(pout);
    const uint64_t t0 = now_ns();
    stage_in(lk, b, self, pin, in_off);
    const uint64_t t1 = now_ns();
    auto* d64 = reinterpret_cast<uint64_t*>(d + in_total);
    auto* dst = reinterpret_cast<int32_t*>(d + in_total + (6 * nb + 1) * 8);
    uint8_t* dslots = d + in_total + arr;
    hipStream_t s = ctx.stream();
    hip_check(hipMemcpyAsync(d, pin, in_total + 3 * nb * 8, hipMemcpyHostToDevice, s), "H2D encode input");
    int st = rpp_encode_batch_ws(&cfg_, reinterpret_cast<uint16_t const*>(d), d64, d64 + nb, static_cast<uint32_t>(nb),
                                 dslots, d64 + 2 * nb, d64 + 3 * nb, dst, total_samples, max_samples, ws, ws_bytes, s);
    if (st != RPP_OK) throw_status(st);
    st = rpp_pack_batch(dslots, d64 + 2 * nb, d64 + 3 * nb, static_cast<uint32_t>(nb), pout_dev, d64 + 4 * nb,
                        d64 + 5 * nb, s);
    if (st != RPP_OK) throw_status(st);
    hip_check(hipMemcpyAsync(pout + out_total, d64 + 3 * nb, arr - 3 * nb * 8, hipMemcpyDeviceToHost, s),
              "D2H encode sizes");
    g_enc_launches.fetch_add(1, std::memory_order_relaxed);
    g_enc_blocks.fetch_add(nb, std::memory_order_relaxed);
    ctx.sync();
    g_stage_ns.fetch_add(t1 - t0, std::memory_order_relaxed);
    g_device_ns.fetch_add(now_ns() - t1, std::memory_order_relaxed);
    auto const* r64 = reinterpret_cast<uint64_t const*>(pout + out_total);  // out_bytes | dst_off | total
    auto const* hst = reinterpret_cast<int32_t const*>(pout + out_total + (3 * nb + 1) * 8);
    for (size_t i = 0; i < nb; ++i) {
      b[i]->status = hst[i];
      b[i]->result_bytes = hst[i] == RPP_OK ? r64[i] : 0;
      b[i]->pin_out = pout + r64[nb + i];
      if (b[i]->status == RPP_OK && b[i]->result_bytes > b[i]->out_cap) b[i]->status = RPP_OUTPUT_TOO_SMALL;
    }
    publish(lk, b, self);
  }

  // One synchronisation per batch: one H2D copy (streams and parameters),
  // one D2H copy (statuses and samples).
  void launch_decode(std::unique_lock<std::mutex>& lk, std::vector<request*> const& b, request& self,
                     device_ctx& ctx) {
    const size_t nb = b.size();
    std::vector<size_t> in_off(nb), out_off(nb);
    size_t in_total = 0, out_total = 0;
    uint64_t total_samples = 0, max_samples = 0;
    for (size_t i = 0; i < nb; ++i) {
      in_off[i] = in_total;
      in_total += align16(b[i]->in_bytes);
      out_off[i] = out_total;
      out_total += align16(b[i]->out_cap);
      total_samples += b[i]->n_samples;
      max_samples = std::max<uint64_t>(max_samples, b[i]->n_samples);
    }
    // device: [in][u64 in_off | in_bytes | out_off | n][i32 status][out samples]
    // pinned in: [in][u64 in_off | in_bytes | out_off | n]   (one H2D copy)
    // pinned out: [i32 status][out samples]                  (one D2H copy)
    const size_t st_bytes = align16(nb * 4);
    uint8_t* d = ctx.dev(in_total + 4 * nb * 8 + st_bytes + out_total + 64);
    uint8_t* pin = ctx.pin_in(in_total + 4 * nb * 8 + 64);
    uint8_t* pout = ctx.pin_out(st_bytes + out_total + 64);
    auto* h64 = reinterpret_cast<uint64_t*>(pin + in_total);
    for (size_t i = 0; i < nb; ++i) {
      h64[i] = in_off[i];
      h64[nb + i] = b[i]->in_bytes;
      h64[2 * nb + i] = out_off[i] / 2;
      h64[3 * nb + i] = b[i]->n_samples;
    }
    // long blocks (16 MiB DwarFS blocks) are parsed in segments by several waves
    const uint64_t ws_bytes = rpp_decode_workspace_bytes(&cfg_, total_samples, max_samples, static_cast<uint32_t>(nb));
    uint8_t* ws = ws_bytes ? ctx.workspace(ws_bytes) : nullptr;
    const uint64_t t0 = now_ns();
    stage_in(lk, b, self, pin, in_off);
    const uint64_t t1 = now_ns();
    auto* d64 = reinterpret_cast<uint64_t*>(d + in_total);
    auto* dst = reinterpret_cast<int32_t*>(d + in_total + 4 * nb * 8);
    uint8_t* dout = d + in_total + 4 * nb * 8 + st_bytes;
    hipStream_t s = ctx.stream();
    hip_check(hipMemcpyAsync(d, pin, in_total + 4 * nb * 8, hipMemcpyHostToDevice, s), "H2D decode input");
    int st = rpp_decode_batch_ws(&cfg_, d, d64, d64 + nb, static_cast<uint32_t>(nb), reinterpret_cast<uint16_t*>(dout),
                                 d64 + 2 * nb, d64 + 3 * nb, dst, total_samples, max_samples, ws, ws_bytes, s);
    if (st != RPP_OK) throw_status(st);
    hip_check(hipMemcpyAsync(pout, dst, st_bytes + out_total, hipMemcpyDeviceToHost, s), "D2H decoded");
    g_dec_launches.fetch_add(1, std::memory_order_relaxed);
    g_dec_blocks.fetch_add(nb, std::memory_order_relaxed);
    ctx.sync();
    g_stage_ns.fetch_add(t1 - t0, std::memory_order_relaxed);
    g_device_ns.fetch_add(now_ns() - t1, std::memory_order_relaxed);
    auto const* hst = reinterpret_cast<int32_t const*>(pout);
    for (size_t i = 0; i < nb; ++i) {
      b[i]->status = hst[i];
      b[i]->result_bytes = hst[i] == RPP_OK ? b[i]->out_cap : 0;
      b[i]->pin_out = pout + st_bytes + out_off[i];
    }
    publish(lk, b, self);
  }

  int dev_;
  rpp_config cfg_;
  bool encode_;
  std::mutex mu_;
  std::deque<request*> pending_;
  int active_ = 0;
};

batch_queue& queue_for(int dev, rpp_config const& c, bool encode) {
  static std::mutex mu;
  static auto* queues = new std::map<std::tuple<int, uint32_t, uint32_t, uint32_t, uint32_t, bool>, batch_queue*>;
  std::lock_guard<std::mutex> lk(mu);
  auto key = std::make_tuple(dev, c.block_size, c.component_stream_count, c.big_endian, c.unused_lsb_count, encode);
  auto it = queues->find(key);
  if (it == queues->end()) it = queues->emplace(key, new batch_queue(dev, c, encode)).first;
  return *it->second;
}

// Runs one request through its queue (the calling thread may become the
// leader of a batch that contains it).
void submit(batch_queue& q, request& r) {
  q.run(r);
  if (r.status == RPP_HIP_ERROR) throw std::runtime_error(r.error.empty() ? "ricepp_amd: HIP error" : r.error);
  if (r.status != RPP_OK) throw_status(r.status);
}

class encoder_impl final : public encoder_interface<uint16_t> {
 public:
  encoder_impl(rpp_config c, int dev) : cfg_{c}, q_{queue_for(dev, c, true)} {}

  size_t worst_case_encoded_bytes(size_t n) const override { return rpp_worst_case_bytes(&cfg_, n); }
  size_t worst_case_encoded_bytes(std::span<uint16_t const> in) const override {
    return worst_case_encoded_bytes(in.size());
  }

  std::vector<uint8_t> encode(std::span<uint16_t const> input) const override {
    std::vector<uint8_t> out(worst_case_encoded_bytes(input.size()));
    auto used = encode(std::span<uint8_t>{out}, input);
    out.resize(used.size());
    return out;
  }

  // ricepp_cpuspecific.cpp:101-108: output must hold the worst case
  std::span<uint8_t> encode(std::span<uint8_t> output, std::span<uint16_t const> input) const override {
    if (output.size() < worst_case_encoded_bytes(input.size()))
      throw std::length_error("ricepp_amd: output smaller than worst_case_encoded_bytes");
    if (input.size() % cfg_.component_stream_count) throw_status(RPP_INVALID_ARGUMENT);
    request r{reinterpret_cast<uint8_t const*>(input.data()), input.size_bytes(), output.data(), output.size(),
              input.size()};
    submit(q_, r);
    return output.subspan(0, r.result_bytes);
  }

 private:
  rpp_config cfg_;
  batch_queue& q_;
};

class decoder_impl final : public decoder_interface<uint16_t> {
 public:
  decoder_impl(rpp_config c, int dev) : cfg_{c}, q_{queue_for(dev, c, false)} {}

  // ricepp_cpuspecific.cpp:127-144: decodes exactly output.size() samples
  void decode(std::span<uint16_t> output, std::span<uint8_t const> input) const override {
    if (output.size() % cfg_.component_stream_count) throw_status(RPP_INVALID_ARGUMENT);
    request r{input.data(), input.size(), reinterpret_cast<uint8_t*>(output.data()), output.size_bytes(),
              output.size()};
    submit(q_, r);
  }

 private:
  rpp_config cfg_;
  batch_queue& q_;
};

// ---- minimal JSON for the flat metadata objects of the plugin ----
// (the reference uses nlohmann::json; only string and integer members occur)
std::map<std::string, std::string> parse_flat_json(std::string const& s) {
  std::map<std::string, std::string> m;
  size_t i = 0;
  auto skip = [&] {
    while (i < s.size() && std::isspace(static_cast<unsigned char>(s[i]))) ++i;
  };
  auto str = [&]() -> std::string {
    std::string r;
    if (i >= s.size() || s[i] != '"') throw std::runtime_error("ricepp_amd: malformed metadata JSON");
    for (++i; i < s.size() && s[i] != '"'; ++i) {
      if (s[i] == '\\' && i + 1 < s.size()) ++i;
      r += s[i];
    }
    ++i;
    return r;
  };
  skip();
  if (i >= s.size() || s[i] != '{') throw std::runtime_error("ricepp_amd: malformed metadata JSON");
  ++i;
  for (;;) {
    skip();
    if (i >= s.size()) throw std::runtime_error("ricepp_amd: malformed metadata JSON");
    if (s[i] == '}') break;
    std::string k = str();
    skip();
    if (i >= s.size() || s[i] != ':') throw std::runtime_error("ricepp_amd: malformed metadata JSON");
    ++i;
    skip();
    std::string v;
    if (i < s.size() && s[i] == '"') {
      v = "\"" + str();
    } else {
      while (i < s.size() && s[i] != ',' && s[i] != '}' && !std::isspace(static_cast<unsigned char>(s[i]))) v += s[i++];
    }
    m[k] = v;
    skip();
    if (i < s.size() && s[i] == ',') ++i;
  }
  return m;
}

int json_int(std::map<std::string, std::string> const& m, char const* key) {
  auto it = m.find(key);
  if (it == m.end() || it->second.empty() || it->second[0] == '"')
    throw std::runtime_error(std::string("ricepp_amd: metadata lacks integer '") + key + "'");
  int v = 0;
  auto r = std::from_chars(it->second.data(), it->second.data() + it->second.size(), v);
  if (r.ec != std::errc{}) throw std::runtime_error(std::string("ricepp_amd: bad integer '") + key + "'");
  return v;
}

std::string json_str(std::map<std::string, std::string> const& m, char const* key) {
  auto it = m.find(key);
  if (it == m.end() || it->second.empty() || it->second[0] != '"')
    throw std::runtime_error(std::string("ricepp_amd: metadata lacks string '") + key + "'");
  return it->second.substr(1);
}

constexpr uint32_t kRiceppVersion = 1;  // src/compression/ricepp.cpp:55

}  // namespace

template <>
std::unique_ptr<encoder_interface<uint16_t>> create_encoder<uint16_t>(codec_config const& config) {
  rpp_config c = to_rpp(config);
  if (rpp_check_config(&c) != RPP_OK) throw std::runtime_error("Unsupported configuration");
  return std::make_unique<encoder_impl>(c, current_device());
}

template <>
std::unique_ptr<decoder_interface<uint16_t>> create_decoder<uint16_t>(codec_config const& config) {
  rpp_config c = to_rpp(config);
  if (rpp_check_config(&c) != RPP_OK) throw std::runtime_error("Unsupported configuration");
  return std::make_unique<decoder_impl>(c, current_device());
}

void inject_context_failures(uint32_t n) { g_ctx_faults.store(n); }

facade_stats get_facade_stats() {
  return facade_stats{g_enc_launches.load(), g_enc_blocks.load(), g_dec_launches.load(), g_dec_blocks.load(),
                      g_ctx_created.load(),     g_stage_ns.load(),   g_device_ns.load(),     g_finish_ns.load()};
}

// ---- block_compressor (src/compression/ricepp.cpp:57-182, 272-296) ----

block_compressor::block_compressor(size_t block_size) : block_size_{block_size} {}

std::unique_ptr<block_compressor> block_compressor::create(std::string const& spec) {
  // "ricepp" or "ricepp:block_size=N" (option_map, default 128, :280); like
  // the reference's factory, the value is not range-checked here
  size_t bs = 128;
  std::string name = spec.substr(0, spec.find(':'));
  if (name != "ricepp") throw std::runtime_error("unknown compression: " + name);
  if (auto c = spec.find(':'); c != std::string::npos) {
    std::string opts = spec.substr(c + 1);
    size_t p = 0;
    while (p < opts.size()) {
      size_t e = opts.find(',', p);
      std::string kv = opts.substr(p, e == std::string::npos ? std::string::npos : e - p);
      auto eq = kv.find('=');
      if (kv.substr(0, eq) != "block_size" || eq == std::string::npos)
        throw std::runtime_error("invalid option(s) for ricepp: " + kv);
      bs = std::stoul(kv.substr(eq + 1));
      if (e == std::string::npos) break;
      p = e + 1;
    }
  }
  return std::make_unique<block_compressor>(bs);
}

std::unique_ptr<block_compressor> block_compressor::clone() const {
  return std::make_unique<block_compressor>(*this);
}

std::string block_compressor::describe() const { return "ricepp [block_size=" + std::to_string(block_size_) + "]"; }

std::string block_compressor::metadata_requirements() const {
  // ricepp.cpp:150-159 (nlohmann::json dump: keys sorted)
  return R"({"bytes_per_sample":["set",[2]],"component_count":["range",1,2],)"
         R"("endianness":["set",["big","little"]],"unused_lsb_count":["range",0,8]})";
}

size_t block_compressor::compression_granularity(std::string const& metadata) const {
  auto m = parse_flat_json(metadata);  // ricepp.cpp:161-173
  return static_cast<size_t>(json_int(m, "component_count") * json_int(m, "bytes_per_sample"));
}

std::vector<uint8_t> block_compressor::compress(std::span<uint8_t const> data, std::string const* metadata) const {
  if (!metadata) throw std::runtime_error("internal error: ricepp compression requires metadata");  // :70-73
  auto meta = parse_flat_json(*metadata);
  auto endianness = json_str(meta, "endianness");
  int component_count = json_int(meta, "component_count");
  int unused_lsb_count = json_int(meta, "unused_lsb_count");
  int bytes_per_sample = json_int(meta, "bytes_per_sample");
  if (bytes_per_sample != 2 || unused_lsb_count < 0 || unused_lsb_count > 8 || component_count < 1 ||
      component_count > 2)
    throw std::runtime_error("ricepp_amd: metadata out of range");  // asserts at :82-84
  if (data.size() % static_cast<size_t>(component_count * bytes_per_sample))  // :86-91
    throw std::runtime_error("unexpected data configuration: " + std::to_string(data.size()) +
                             " bytes to compress, " + std::to_string(component_count) + " components, " +
                             std::to_string(bytes_per_sample) + " bytes per sample");
  auto const byteorder = endianness == "big" ? std::endian::big : std::endian::little;
  // :97-102 -- throws "Unsupported configuration" for an unsupported block size
  auto enc = create_encoder<uint16_t>({
      .block_size = block_size_,
      .component_stream_count = static_cast<size_t>(component_count),
      .byteorder = byteorder,
      .unused_lsb_count = static_cast<unsigned>(unused_lsb_count),
  });
  rpp_frame f{data.size(), static_cast<uint32_t>(block_size_), static_cast<uint32_t>(component_count),
              static_cast<uint32_t>(bytes_per_sample), static_cast<uint32_t>(unused_lsb_count),
              byteorder == std::endian::big ? 1u : 0u, kRiceppVersion};
  std::vector<uint8_t> out(64);
  size_t hdr = rpp_frame_header(&f, out.data());
  size_t n = data.size() / 2;
  out.resize(hdr + enc->worst_case_encoded_bytes(n));
  // (the samples are read in place: the staging copy handles any alignment)
  std::span<uint16_t const> samples{reinterpret_cast<uint16_t const*>(data.data()), n};
  auto used = enc->encode(std::span<uint8_t>{out}.subspan(hdr), samples);
  out.resize(hdr + used.size());
  out.shrink_to_fit();
  return out;
}

// ---- block_decompressor (src/compression/ricepp.cpp:184-255) ----

block_decompressor::block_decompressor(std::span<uint8_t const> data) {
  long h = rpp_parse_frame(data.data(), data.size(), &frame_);
  if (h < 0) throw std::runtime_error("ricepp_amd: malformed ricepp block header");
  data_ = data.subspan(static_cast<size_t>(h));
  if (frame_.ricepp_version > kRiceppVersion)  // :243-247
    throw std::runtime_error("[RICEPP] unsupported version: " + std::to_string(frame_.ricepp_version));
  decoder_ = create_decoder<uint16_t>({
      .block_size = frame_.block_size,
      .component_stream_count = frame_.component_count,
      .byteorder = frame_.big_endian ? std::endian::big : std::endian::little,
      .unused_lsb_count = frame_.unused_lsb_count,
  });
  if (frame_.bytes_per_sample != 2)  // :196-200
    throw std::runtime_error("[RICEPP] unsupported bytes per sample: " + std::to_string(frame_.bytes_per_sample));
}

std::optional<std::string> block_decompressor::metadata() const {
  // :203-212 (nlohmann::json dump: keys sorted)
  return std::string(R"({"bytes_per_sample":)") + std::to_string(frame_.bytes_per_sample) +
         R"(,"component_count":)" + std::to_string(frame_.component_count) + R"(,"endianness":")" +
         (frame_.big_endian ? "big" : "little") + R"(","unused_lsb_count":)" +
         std::to_string(frame_.unused_lsb_count) + "}";
}

void block_decompressor::start_decompression(std::vector<uint8_t>* target) {
  target_ = target;
  target_->reserve(frame_.uncompressed_bytes);  // src/compression/base.cpp:37-51
}

bool block_decompressor::decompress_frame(size_t) {
  if (!target_) throw std::runtime_error("decompression not started");  // :216
  if (!decoder_) return false;
  target_->resize(frame_.uncompressed_bytes);
  std::span<uint16_t> out{reinterpret_cast<uint16_t*>(target_->data()), target_->size() / 2};
  decoder_->decode(out, data_);
  decoder_.reset();
  return true;
}

std::vector<uint8_t> block_decompressor::decompress(std::span<uint8_t const> data) {
  block_decompressor d{data};
  std::vector<uint8_t> out;
  d.start_decompression(&out);
  d.decompress_frame(d.uncompressed_size());
  return out;
}

// ---- pcm_sample_transformer (src/pcm_sample_transformer.cpp:372-377) ----

pcm_sample_transformer::pcm_sample_transformer(pcm_sample_endianness end, pcm_sample_signedness sig,
                                               pcm_sample_padding pad, int bytes, int bits) {
  fmt_.big_endian = end == pcm_sample_endianness::Big ? 1u : 0u;
  fmt_.is_signed = sig == pcm_sample_signedness::Signed ? 1u : 0u;
  fmt_.lsb_padded = pad == pcm_sample_padding::Lsb ? 1u : 0u;
  fmt_.bytes = bytes < 0 ? 0u : static_cast<uint32_t>(bytes);
  fmt_.bits = bits < 0 ? 0u : static_cast<uint32_t>(bits);
  const int st = rpp_pcm_check_format(&fmt_);
  if (st == RPP_UNSUPPORTED_CONFIG || bytes < 1 || bytes > 4)
    throw std::runtime_error("unsupported number of bytes per sample: " + std::to_string(bytes));
  if (st != RPP_OK) throw std::invalid_argument("pcm_sample_transformer: bits outside 1..8*bytes");
  device_ = current_device();
}

pcm_sample_transformer::~pcm_sample_transformer() = default;
pcm_sample_transformer::pcm_sample_transformer(pcm_sample_transformer&&) noexcept = default;
pcm_sample_transformer& pcm_sample_transformer::operator=(pcm_sample_transformer&&) noexcept = default;

void pcm_sample_transformer::unpack(std::span<int32_t> dst, std::span<uint8_t const> src) const {
  if (src.size() != fmt_.bytes * dst.size()) throw std::invalid_argument("pcm unpack: src.size() != bytes * dst.size()");
  if (dst.empty()) return;
  const size_t off_out = align16(src.size());
  device_guard g{device_};
  ctx_lease ctx{device_};
  uint8_t* d = ctx->dev(off_out + dst.size_bytes());
  hipStream_t s = ctx->stream();
  hip_check(hipMemcpyAsync(d, src.data(), src.size(), hipMemcpyHostToDevice, s), "H2D pcm");
  const int st = rpp_pcm_unpack(&fmt_, d, reinterpret_cast<int32_t*>(d + off_out), dst.size(), s);
  if (st != RPP_OK) throw_status(st);
  hip_check(hipMemcpyAsync(dst.data(), d + off_out, dst.size_bytes(), hipMemcpyDeviceToHost, s), "D2H pcm");
  ctx->sync();
}

void pcm_sample_transformer::pack(std::span<uint8_t> dst, std::span<int32_t const> src) const {
  if (dst.size() != fmt_.bytes * src.size()) throw std::invalid_argument("pcm pack: dst.size() != bytes * src.size()");
  if (src.empty()) return;
  const size_t off_out = align16(src.size_bytes());
  device_guard g{device_};
  ctx_lease ctx{device_};
  uint8_t* d = ctx->dev(off_out + dst.size());
  hipStream_t s = ctx->stream();
  hip_check(hipMemcpyAsync(d, src.data(), src.size_bytes(), hipMemcpyHostToDevice, s), "H2D pcm");
  const int st = rpp_pcm_pack(&fmt_, reinterpret_cast<int32_t const*>(d), d + off_out, src.size(), s);
  if (st != RPP_OK) throw_status(st);
  hip_check(hipMemcpyAsync(dst.data(), d + off_out, dst.size(), hipMemcpyDeviceToHost, s), "D2H pcm");
  ctx->sync();
}

}  // namespace ricepp_amd
