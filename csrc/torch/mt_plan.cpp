// Device-resident multi-tensor launch tables, cached by tensor addresses.
//
// A list passed with the same addresses again (parameters, optimizer state) gets
// its table (TensorDesc[] + ChunkDesc[]) built and uploaded once and re-used: zero
// metadata traffic per step, and the launch stays valid under hipGraph capture
// after one warm-up call.  Gradient lists change addresses every step (Apex sets
// grads to None between steps, autograd re-allocates them): those are never
// entered in the address cache; their chunk list comes from a cache keyed by the
// tensor sizes and only the tensor table (pointers) is uploaded per call, through
// a pinned staging ring allocated once (mt_plan.cpp: measured 2-5 new plans per
// step before, each a pinned allocation + a full chunk-table upload).
#include <cstdlib>
#include <cstring>
#include <list>
#include <mutex>
#include <unordered_map>

#include <c10/hip/HIPException.h>
#include <c10/hip/HIPGraphsC10Utils.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "common.h"

namespace amd {

namespace {

struct Key {
  std::vector<uint64_t> words;
  bool operator==(const Key& o) const { return words == o.words; }
};
struct KeyHash {
  size_t operator()(const Key& k) const {
    uint64_t h = 1469598103934665603ull;
    for (uint64_t w : k.words) {
      h ^= w;
      h *= 1099511628211ull;
    }
    return (size_t)h;
  }
};

struct Cache {
  std::mutex mu;
  std::list<Key> lru;  // front = most recent
  struct Entry {
    MTPlan plan;
    std::list<Key>::iterator pos;
  };
  std::unordered_map<Key, Entry, KeyHash> map;
  static constexpr size_t kMax = 512;
};

Cache& cache() {
  static Cache c;
  return c;
}

// Same memory order of elements (strides of size-1 dims are irrelevant).
bool same_layout(const at::Tensor& a, const at::Tensor& b) {
  if (a.dim() != b.dim()) return a.is_contiguous() && b.is_contiguous();
  for (int64_t k = 0; k < a.dim(); ++k) {
    if (a.size(k) != b.size(k)) return false;
    if (a.size(k) > 1 && a.stride(k) != b.stride(k)) return false;
  }
  return true;
}

}  // namespace

bool mt_validate(const TensorLists& lists, int min_depth, int max_depth) {
  TORCH_CHECK((int)lists.size() >= min_depth && (int)lists.size() <= max_depth,
              "expected between ", min_depth, " and ", max_depth, " tensor lists, got ",
              lists.size());
  const size_t n = lists[0].size();
  bool on_gpu = false;
  bool first = true;
  for (size_t d = 0; d < lists.size(); ++d) {
    TORCH_CHECK(lists[d].size() == n, "tensor list ", d, " has ", lists[d].size(),
                " tensors, expected ", n);
    for (size_t i = 0; i < n; ++i) {
      const at::Tensor& t = lists[d][i];
      // Elementwise ops only need a dense block whose element order matches across
      // the lists: contiguous, or e.g. channels_last weights with identical strides
      // in every slot (grads, masters and state are created with preserved format).
      TORCH_CHECK(t.is_non_overlapping_and_dense() && same_layout(t, lists[0][i]),
                  "multi_tensor ops need dense tensors with matching strides (list ", d,
                  ", index ", i, ")");
      TORCH_CHECK(t.numel() == lists[0][i].numel(), "size mismatch at list ", d, " index ", i);
      if (first) {
        on_gpu = t.is_cuda();
        first = false;
      } else {
        TORCH_CHECK(t.is_cuda() == on_gpu, "all tensors must be on the same device type");
      }
    }
  }
  return on_gpu;
}

namespace {

// Per-call tensor tables travel through one pinned staging ring allocated once
// (hipHostMalloc) instead of a pinned tensor per plan: a fresh pinned allocation
// can stall the host behind the device, and gradient lists change addresses every
// step (Apex's grad-to-None elision re-allocates them), so those plans are built
// every step.  A region is reused only after the copy that read it has completed.
struct PinnedRing {
  uint8_t* base = nullptr;
  size_t cap = 0, head = 0;
  struct Use {
    size_t b, e;
    hipEvent_t ev;
  };
  std::list<Use> inflight;  // issue order
  std::vector<hipEvent_t> spare;
  static constexpr size_t kCap = (size_t)16 << 20;

  bool ok() {
    if (!base) {
      if (hipHostMalloc((void**)&base, kCap, hipHostMallocDefault) != hipSuccess) {
        base = nullptr;
        return false;
      }
      cap = kCap;
    }
    return true;
  }
  // stage `bytes` from src and copy them to dst on stream st
  void upload(void* dst, const void* src, size_t bytes, hipStream_t st) {
    const size_t need = (bytes + 255) / 256 * 256;
    if (need > cap) {  // larger than the whole ring: a synchronous copy
      C10_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
      C10_HIP_CHECK(hipStreamSynchronize(st));
      return;
    }
    if (head + need > cap) head = 0;
    const size_t b = head, e = head + need;
    // wait for (normally long finished) copies that read the region we overwrite
    for (auto it = inflight.begin(); it != inflight.end();) {
      if (it->b < e && b < it->e) {
        C10_HIP_CHECK(hipEventSynchronize(it->ev));
        spare.push_back(it->ev);
        it = inflight.erase(it);
      } else {
        ++it;
      }
    }
    std::memcpy(base + b, src, bytes);
    C10_HIP_CHECK(hipMemcpyAsync(dst, base + b, bytes, hipMemcpyHostToDevice, st));
    hipEvent_t ev;
    if (!spare.empty()) {
      ev = spare.back();
      spare.pop_back();
    } else {
      C10_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    C10_HIP_CHECK(hipEventRecord(ev, st));
    inflight.push_back(Use{b, e, ev});
    head = e;
  }
};

PinnedRing& ring() {
  static PinnedRing r;
  return r;
}

// chunk tables keyed by (device, tensor sizes): a list whose addresses change
// every step keeps its sizes
struct ChunkCache {
  std::unordered_map<Key, at::Tensor, KeyHash> map;
  static constexpr size_t kMax = 256;
};
ChunkCache& chunk_cache() {
  static ChunkCache c;
  return c;
}

// keys seen once: a list seen a second time gets a fully cached plan
struct SeenSet {
  std::list<Key> order;
  static constexpr size_t kMax = 64;
  bool check_and_add(const Key& k) {
    for (auto it = order.begin(); it != order.end(); ++it)
      if (*it == k) {
        order.erase(it);
        return true;
      }
    order.push_front(k);
    if (order.size() > kMax) order.pop_back();
    return false;
  }
};
SeenSet& seen() {
  static SeenSet s;
  return s;
}

// tensor table always; the chunk list only when `chunks` is given
int64_t build_tables(const TensorLists& lists, std::vector<TensorDesc>& tds,
                     std::vector<ChunkDesc>* chunks) {
  const int depth = (int)lists.size();
  const int n = (int)lists[0].size();
  tds.resize((size_t)n);
  int64_t total = 0;
  for (int i = 0; i < n; ++i) {
    TensorDesc& td = tds[(size_t)i];
    std::memset(&td, 0, sizeof(td));
    td.numel = lists[0][i].numel();
    int aligned = 1;
    for (int d = 0; d < depth; ++d) {
      void* p = lists[d][i].data_ptr();
      td.ptr[d] = p;
      if (((uintptr_t)p) % 16 != 0) aligned = 0;
    }
    td.aligned = aligned;
    td.first_chunk = (int32_t)total;
    const int64_t nch = (td.numel + kTile - 1) / kTile;
    if (chunks)
      for (int64_t k = 0; k < nch; ++k) chunks->push_back(ChunkDesc{i, (int32_t)k});
    total += nch;
  }
  TORCH_CHECK(total < (int64_t)INT32_MAX, "too many chunks");
  return total;
}

}  // namespace

MTPlan mt_plan(const TensorLists& lists) {
  const int depth = (int)lists.size();
  const int n = (int)lists[0].size();
  TORCH_CHECK(depth <= kMaxDepth, "depth > kMaxDepth");
  Key key;
  key.words.reserve(2 + (size_t)n * (depth + 1));
  key.words.push_back((uint64_t)depth);
  key.words.push_back((uint64_t)n);
  for (int i = 0; i < n; ++i) {
    key.words.push_back((uint64_t)lists[0][i].numel());
    for (int d = 0; d < depth; ++d) key.words.push_back((uint64_t)lists[d][i].data_ptr());
  }
  Cache& c = cache();
  std::lock_guard<std::mutex> g(c.mu);
  auto it = c.map.find(key);
  if (it != c.map.end()) {
    c.lru.splice(c.lru.begin(), c.lru, it->second.pos);
    // a table referenced by a captured graph must outlive the graph: pin it
    if (c10::hip::currentStreamCaptureStatusMayInitCtx() != c10::hip::CaptureStatus::None)
      it->second.plan.captured = true;
    return it->second.plan;
  }

  auto dev = lists[0][0].device();
  const bool capturing =
      c10::hip::currentStreamCaptureStatusMayInitCtx() != c10::hip::CaptureStatus::None;
  hipStream_t st = c10::hip::getCurrentHIPStream().stream();

  if (!capturing && !seen().check_and_add(key) && ring().ok()) {
    // First sighting of these addresses: chunk list from the size-keyed cache, the
    // tensor table uploaded for this call only (nothing enters the address cache).
    Key skey;
    skey.words.reserve(3 + (size_t)n);
    skey.words.push_back((uint64_t)dev.index());
    skey.words.push_back((uint64_t)n);
    for (int i = 0; i < n; ++i) skey.words.push_back((uint64_t)lists[0][i].numel());
    std::vector<TensorDesc> tds;
    ChunkCache& cc = chunk_cache();
    auto cit = cc.map.find(skey);
    const int64_t nchunks = build_tables(lists, tds, nullptr);
    if (cit == cc.map.end()) {
      std::vector<ChunkDesc> chunks;
      chunks.reserve((size_t)nchunks);
      std::vector<TensorDesc> unused;
      build_tables(lists, unused, &chunks);
      if (cc.map.size() >= ChunkCache::kMax) {
        for (auto& kv : cc.map) kv.second.record_stream(at::hip::getCurrentHIPStreamMasqueradingAsCUDA());
        cc.map.clear();
      }
      const size_t cbytes = chunks.size() * sizeof(ChunkDesc) + 16;
      at::Tensor ct = at::empty({(int64_t)cbytes}, at::TensorOptions().dtype(at::kByte).device(dev));
      if (!chunks.empty()) ring().upload(ct.data_ptr(), chunks.data(), chunks.size() * sizeof(ChunkDesc), st);
      cit = cc.map.emplace(skey, ct).first;
    }
    const size_t tbytes = tds.size() * sizeof(TensorDesc);
    MTPlan plan;
    plan.table = at::empty({(int64_t)(tbytes + 16)}, at::TensorOptions().dtype(at::kByte).device(dev));
    if (tbytes) ring().upload(plan.table.data_ptr(), tds.data(), tbytes, st);
    plan.chunks = cit->second;
    plan.L.tensors = reinterpret_cast<const TensorDesc*>(plan.table.data_ptr<uint8_t>());
    plan.L.chunks = reinterpret_cast<const ChunkDesc*>(plan.chunks.data_ptr<uint8_t>());
    plan.L.ntensors = n;
    plan.L.nchunks = (int32_t)nchunks;
    return plan;
  }

  // Build the host image.
  std::vector<TensorDesc> tds;
  std::vector<ChunkDesc> chunks;
  build_tables(lists, tds, &chunks);
  const size_t tbytes = tds.size() * sizeof(TensorDesc);
  const size_t cbytes = chunks.size() * sizeof(ChunkDesc);
  const size_t coff = (tbytes + 255) / 256 * 256;
  const size_t total = coff + cbytes + 16;

  at::Tensor table = at::empty({(int64_t)total}, at::TensorOptions().dtype(at::kByte).device(dev));
  at::Tensor host;
  if (!capturing && ring().ok()) {
    // eager: one async copy through the pinned staging ring (no pinned allocation)
    std::vector<uint8_t> img(total, 0);
    if (tbytes) std::memcpy(img.data(), tds.data(), tbytes);
    if (cbytes) std::memcpy(img.data() + coff, chunks.data(), cbytes);
    ring().upload(table.data_ptr(), img.data(), total, st);
  } else if (!capturing) {
    // eager: one async copy from a pinned image kept alive with the plan
    host = at::empty({(int64_t)total}, at::TensorOptions().dtype(at::kByte).pinned_memory(true));
    uint8_t* hp = host.data_ptr<uint8_t>();
    std::memset(hp, 0, total);
    if (tbytes) std::memcpy(hp, tds.data(), tbytes);
    if (cbytes) std::memcpy(hp + coff, chunks.data(), cbytes);
    C10_HIP_CHECK(hipMemcpyAsync(table.data_ptr(), hp, total, hipMemcpyHostToDevice, st));
  } else {
    // inside a hipGraph capture no pinned allocation is allowed: the image
    // travels in kernel arguments, captured by value into the graph
    std::vector<uint8_t> img(total, 0);
    if (tbytes) std::memcpy(img.data(), tds.data(), tbytes);
    if (cbytes) std::memcpy(img.data() + coff, chunks.data(), cbytes);
    upload_by_args(table.data_ptr(), img.data(), total, st);
  }

  MTPlan plan;
  plan.table = table;
  plan.host = host;
  plan.captured = capturing;
  uint8_t* base = table.data_ptr<uint8_t>();
  plan.L.tensors = reinterpret_cast<const TensorDesc*>(base);
  plan.L.chunks = reinterpret_cast<const ChunkDesc*>(base + coff);
  plan.L.ntensors = n;
  plan.L.nchunks = (int32_t)chunks.size();

  if (c.map.size() >= Cache::kMax) {
    // Evict the least recently used table that no captured graph refers to;
    // kernels that may still read it run on the current stream, so tie its
    // lifetime to that stream.
    for (auto it2 = c.lru.end(); it2 != c.lru.begin();) {
      --it2;
      auto oit = c.map.find(*it2);
      if (oit == c.map.end() || oit->second.plan.captured) continue;
      // (the allocator files HIP streams under the CUDA device type: a plain
      // c10::hip stream here is rejected by Tensor::record_stream)
      oit->second.plan.table.record_stream(at::hip::getCurrentHIPStreamMasqueradingAsCUDA());
      c.map.erase(oit);
      c.lru.erase(it2);
      break;
    }
  }
  c.lru.push_front(key);
  auto res = c.map.emplace(key, Cache::Entry{plan, c.lru.begin()});
  return res.first->second.plan;
}

void mt_plan_cache_clear() {
  Cache& c = cache();
  std::lock_guard<std::mutex> g(c.mu);
  c.map.clear();
  c.lru.clear();
  chunk_cache().map.clear();
  seen().order.clear();
}

int64_t mt_plan_cache_size() {
  Cache& c = cache();
  std::lock_guard<std::mutex> g(c.mu);
  return (int64_t)c.map.size();
}

}  // namespace amd
