// libgpupool_share.so — isolation for time-shared MI355X GPUs (the HAMi layer of the reference
// platform, GPU调度平台搭建.md:289-298: per-sharer memory and compute limits on one GPU).
//
// Loaded into a pod's processes by the ROCm runtime itself: the device plugin's Allocate sets
// HSA_TOOLS_LIB=<this library>, and ROCr calls OnLoad() with its HSA API dispatch table before
// the application makes its first HIP call. Every HIP path ends in a handful of HSA entry points,
// so wrapping those covers hipMalloc / hipMallocAsync / hipMallocManaged / hipExtMallocWithFlags /
// hipMemCreate (VMM) and every stream, including the null stream, without touching HIP:
//
//   * HBM budget (GPUPOOL_HBM_LIMIT_BYTES, per GPU): hsa_amd_memory_pool_allocate and
//     hsa_amd_vmem_handle_create on a GPU-located pool fail with OUT_OF_RESOURCES once the
//     process's live VRAM on that GPU would exceed the budget (HIP reports hipErrorOutOfMemory);
//     hsa_amd_memory_pool_free / hsa_amd_vmem_handle_release return the bytes. The pool SIZE and
//     the agent's MEMORY_AVAIL report the budget, so hipMemGetInfo / torch.cuda.mem_get_info and
//     the caching allocators that size themselves from it see the slot, not the whole GPU.
//   * CU share (GPUPOOL_CU_MASK, CU-mask bit ranges like "0-63" or "0-31,128-159"): every HSA
//     queue created on a GPU gets hsa_amd_queue_cu_set_mask(mask), and an application's own
//     hipExtStreamCreateWithCUMask mask is intersected with it — waves of this process can only
//     be dispatched to the slot's CUs.
//
// Budgets are per process (a pod's rank on its slot); the agent gives sibling slots disjoint CU
// ranges and budgets that sum to at most the GPU's HBM.
#define AMD_INTERNAL_BUILD  // hsa_api_trace.h: include the sibling headers of /opt/rocm/include/hsa
#include <hsa/hsa.h>
#include <hsa/hsa_api_trace.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

struct State {
  std::mutex mu;
  CoreApiTable real_core{};
  AmdExtTable real_amd{};
  uint64_t limit = 0;                       // bytes per GPU; 0 = no budget
  std::vector<uint32_t> mask;               // CU mask words; empty = no mask
  uint32_t mask_bits = 0;
  bool debug = false;
  bool pools_mapped = false;
  std::map<uint64_t, uint64_t> pool_agent;  // GPU-located pool handle -> agent handle
  std::map<uint64_t, uint64_t> used;        // agent handle -> live bytes
  std::unordered_map<void*, std::pair<uint64_t, uint64_t>> ptrs;       // ptr -> (agent, bytes)
  std::unordered_map<uint64_t, std::pair<uint64_t, uint64_t>> vmem;    // handle -> (agent, bytes)
  std::atomic<uint64_t> denied{0}, queues_masked{0}, peak{0};
};

State& st() {
  static State* s = new State();  // never destroyed: HSA may call in during process exit
  return *s;
}

uint64_t parse_bytes(const char* v) {
  if (!v || !*v) return 0;
  char* end = nullptr;
  double x = std::strtod(v, &end);
  std::string suf = end ? end : "";
  double mul = 1;
  if (suf == "Ki" || suf == "K" || suf == "k") mul = 1024.0;
  else if (suf == "Mi" || suf == "M") mul = 1024.0 * 1024;
  else if (suf == "Gi" || suf == "G") mul = 1024.0 * 1024 * 1024;
  else if (suf == "Ti" || suf == "T") mul = 1024.0 * 1024 * 1024 * 1024;
  return static_cast<uint64_t>(x * mul);
}

// "0-63,128-159" -> bit words (32 bits each); bits counted up to the highest set bit, rounded up to
// a multiple of 32 as hsa_amd_queue_cu_set_mask requires.
std::vector<uint32_t> parse_mask(const char* v, uint32_t* bits) {
  std::vector<uint32_t> words;
  *bits = 0;
  if (!v || !*v) return words;
  std::string s(v);
  size_t pos = 0;
  while (pos < s.size()) {
    size_t comma = s.find(',', pos);
    std::string part = s.substr(pos, comma == std::string::npos ? std::string::npos : comma - pos);
    pos = comma == std::string::npos ? s.size() : comma + 1;
    if (part.empty()) continue;
    size_t dash = part.find('-');
    long lo = std::strtol(part.c_str(), nullptr, 10);
    long hi = dash == std::string::npos ? lo : std::strtol(part.c_str() + dash + 1, nullptr, 10);
    if (lo < 0 || hi < lo || hi > 4095) continue;
    for (long b = lo; b <= hi; ++b) {
      size_t w = static_cast<size_t>(b) / 32;
      if (words.size() <= w) words.resize(w + 1, 0);
      words[w] |= 1u << (b % 32);
    }
  }
  *bits = static_cast<uint32_t>(words.size() * 32);
  return words;
}

hsa_status_t collect_pool(hsa_amd_memory_pool_t pool, void* agent_handle) {
  State& s = st();
  hsa_amd_memory_pool_location_t loc{};
  if (s.real_amd.hsa_amd_memory_pool_get_info_fn &&
      s.real_amd.hsa_amd_memory_pool_get_info_fn(pool, HSA_AMD_MEMORY_POOL_INFO_LOCATION, &loc) == HSA_STATUS_SUCCESS &&
      loc == HSA_AMD_MEMORY_POOL_LOCATION_GPU)
    s.pool_agent[pool.handle] = *static_cast<uint64_t*>(agent_handle);
  return HSA_STATUS_SUCCESS;
}

hsa_status_t collect_agent(hsa_agent_t agent, void*) {
  State& s = st();
  hsa_device_type_t type{};
  if (s.real_core.hsa_agent_get_info_fn(agent, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS ||
      type != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  uint64_t h = agent.handle;
  s.used.emplace(h, 0);
  if (s.real_amd.hsa_amd_agent_iterate_memory_pools_fn)
    s.real_amd.hsa_amd_agent_iterate_memory_pools_fn(agent, collect_pool, &h);
  return HSA_STATUS_SUCCESS;
}

// pool -> its GPU agent (0 if the pool is not GPU memory). Caller holds s.mu.
uint64_t agent_of(hsa_amd_memory_pool_t pool) {
  State& s = st();
  if (!s.pools_mapped) {
    s.pools_mapped = true;
    if (s.real_core.hsa_iterate_agents_fn) s.real_core.hsa_iterate_agents_fn(collect_agent, nullptr);
  }
  auto it = s.pool_agent.find(pool.handle);
  return it == s.pool_agent.end() ? 0 : it->second;
}

// Reserve ``size`` bytes on the pool's GPU; false when over budget. Caller holds s.mu.
bool charge(uint64_t agent, size_t size) {
  State& s = st();
  uint64_t& u = s.used[agent];
  if (s.limit && u + size > s.limit) {
    s.denied.fetch_add(1);
    if (s.debug)
      std::fprintf(stderr, "[gpupool-share] deny %zu B: %llu in use of %llu\n", size,
                   static_cast<unsigned long long>(u), static_cast<unsigned long long>(s.limit));
    return false;
  }
  u += size;
  uint64_t pk = s.peak.load();
  while (u > pk && !s.peak.compare_exchange_weak(pk, u)) {}
  return true;
}

hsa_status_t w_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t flags, void** ptr) {
  State& s = st();
  uint64_t agent = 0;
  {
    std::lock_guard<std::mutex> g(s.mu);
    agent = agent_of(pool);
    if (agent && !charge(agent, size)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  hsa_status_t r = s.real_amd.hsa_amd_memory_pool_allocate_fn(pool, size, flags, ptr);
  std::lock_guard<std::mutex> g(s.mu);
  if (!agent) return r;
  if (r == HSA_STATUS_SUCCESS && ptr && *ptr) s.ptrs[*ptr] = {agent, size};
  else s.used[agent] -= size;
  return r;
}

hsa_status_t w_pool_free(void* ptr) {
  State& s = st();
  {
    std::lock_guard<std::mutex> g(s.mu);
    auto it = s.ptrs.find(ptr);
    if (it != s.ptrs.end()) {
      s.used[it->second.first] -= it->second.second;
      s.ptrs.erase(it);
    }
  }
  return s.real_amd.hsa_amd_memory_pool_free_fn(ptr);
}

hsa_status_t w_vmem_create(hsa_amd_memory_pool_t pool, size_t size, hsa_amd_memory_type_t type, uint64_t flags,
                           hsa_amd_vmem_alloc_handle_t* handle) {
  State& s = st();
  uint64_t agent = 0;
  {
    std::lock_guard<std::mutex> g(s.mu);
    agent = agent_of(pool);
    if (agent && !charge(agent, size)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  hsa_status_t r = s.real_amd.hsa_amd_vmem_handle_create_fn(pool, size, type, flags, handle);
  std::lock_guard<std::mutex> g(s.mu);
  if (!agent) return r;
  if (r == HSA_STATUS_SUCCESS && handle) s.vmem[handle->handle] = {agent, size};
  else s.used[agent] -= size;
  return r;
}

hsa_status_t w_vmem_release(hsa_amd_vmem_alloc_handle_t handle) {
  State& s = st();
  {
    std::lock_guard<std::mutex> g(s.mu);
    auto it = s.vmem.find(handle.handle);
    if (it != s.vmem.end()) {
      s.used[it->second.first] -= it->second.second;
      s.vmem.erase(it);
    }
  }
  return s.real_amd.hsa_amd_vmem_handle_release_fn(handle);
}

hsa_status_t w_pool_get_info(hsa_amd_memory_pool_t pool, hsa_amd_memory_pool_info_t attr, void* value) {
  State& s = st();
  hsa_status_t r = s.real_amd.hsa_amd_memory_pool_get_info_fn(pool, attr, value);
  if (r != HSA_STATUS_SUCCESS || attr != HSA_AMD_MEMORY_POOL_INFO_SIZE || !s.limit || !value) return r;
  std::lock_guard<std::mutex> g(s.mu);
  if (agent_of(pool)) {
    size_t* sz = static_cast<size_t*>(value);
    *sz = std::min<size_t>(*sz, static_cast<size_t>(s.limit));
  }
  return r;
}

hsa_status_t w_agent_get_info(hsa_agent_t agent, hsa_agent_info_t attr, void* value) {
  State& s = st();
  hsa_status_t r = s.real_core.hsa_agent_get_info_fn(agent, attr, value);
  if (r != HSA_STATUS_SUCCESS || !s.limit || !value ||
      static_cast<int>(attr) != static_cast<int>(HSA_AMD_AGENT_INFO_MEMORY_AVAIL))
    return r;
  std::lock_guard<std::mutex> g(s.mu);
  auto it = s.used.find(agent.handle);
  if (it != s.used.end()) {
    uint64_t* avail = static_cast<uint64_t*>(value);
    uint64_t left = s.limit > it->second ? s.limit - it->second : 0;
    *avail = std::min(*avail, left);
  }
  return r;
}

bool is_gpu(hsa_agent_t agent) {
  hsa_device_type_t type{};
  return st().real_core.hsa_agent_get_info_fn(agent, HSA_AGENT_INFO_DEVICE, &type) == HSA_STATUS_SUCCESS &&
         type == HSA_DEVICE_TYPE_GPU;
}

hsa_status_t w_queue_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                            void (*callback)(hsa_status_t, hsa_queue_t*, void*), void* data,
                            uint32_t private_segment_size, uint32_t group_segment_size, hsa_queue_t** queue) {
  State& s = st();
  hsa_status_t r = s.real_core.hsa_queue_create_fn(agent, size, type, callback, data, private_segment_size,
                                                   group_segment_size, queue);
  if (r == HSA_STATUS_SUCCESS && queue && *queue && !s.mask.empty() && is_gpu(agent)) {
    hsa_status_t m = s.real_amd.hsa_amd_queue_cu_set_mask_fn(*queue, s.mask_bits, s.mask.data());
    if (m == HSA_STATUS_SUCCESS || static_cast<int>(m) == static_cast<int>(HSA_STATUS_CU_MASK_REDUCED))
      s.queues_masked.fetch_add(1);
    if (s.debug) std::fprintf(stderr, "[gpupool-share] queue %p CU mask (%u bits): status %d\n",
                              static_cast<void*>(*queue), s.mask_bits, static_cast<int>(m));
  }
  return r;
}

hsa_status_t w_queue_cu_set_mask(const hsa_queue_t* queue, uint32_t bits, const uint32_t* mask) {
  // the application's own mask (hipExtStreamCreateWithCUMask) can only narrow the slot's
  State& s = st();
  if (s.mask.empty()) return s.real_amd.hsa_amd_queue_cu_set_mask_fn(queue, bits, mask);
  std::vector<uint32_t> m(s.mask);
  if (bits > 0 && mask) {
    for (size_t i = 0; i < m.size(); ++i) m[i] &= i < bits / 32 ? mask[i] : 0u;
    if (std::all_of(m.begin(), m.end(), [](uint32_t w) { return w == 0; })) m = s.mask;
  }
  return s.real_amd.hsa_amd_queue_cu_set_mask_fn(queue, s.mask_bits, m.data());
}

}  // namespace

extern "C" {

// ROCr tools-library entry point (HSA_TOOLS_LIB): install the wrappers into the dispatch table.
__attribute__((visibility("default"))) bool OnLoad(HsaApiTable* table, uint64_t runtime_version,
                                                   uint64_t failed_tool_count, const char* const* failed_tool_names) {
  if (!table || !table->core_ || !table->amd_ext_) return false;
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  s.real_core = *table->core_;
  s.real_amd = *table->amd_ext_;
  s.limit = parse_bytes(std::getenv("GPUPOOL_HBM_LIMIT_BYTES"));
  s.mask = parse_mask(std::getenv("GPUPOOL_CU_MASK"), &s.mask_bits);
  const char* dbg = std::getenv("GPUPOOL_SHARE_DEBUG");
  s.debug = dbg && *dbg && *dbg != '0';
  if (s.limit) {
    table->amd_ext_->hsa_amd_memory_pool_allocate_fn = w_pool_allocate;
    table->amd_ext_->hsa_amd_memory_pool_free_fn = w_pool_free;
    table->amd_ext_->hsa_amd_vmem_handle_create_fn = w_vmem_create;
    table->amd_ext_->hsa_amd_vmem_handle_release_fn = w_vmem_release;
    table->amd_ext_->hsa_amd_memory_pool_get_info_fn = w_pool_get_info;
    table->core_->hsa_agent_get_info_fn = w_agent_get_info;
  }
  if (!s.mask.empty()) {
    table->core_->hsa_queue_create_fn = w_queue_create;
    table->amd_ext_->hsa_amd_queue_cu_set_mask_fn = w_queue_cu_set_mask;
  }
  if (s.debug)
    std::fprintf(stderr, "[gpupool-share] loaded: HBM limit %llu B per GPU, CU mask %u bits\n",
                 static_cast<unsigned long long>(s.limit), s.mask_bits);
  return true;
}

__attribute__((visibility("default"))) void OnUnload() {}

// Counters for tests and diagnostics: JSON into buf.
__attribute__((visibility("default"))) int gpupool_share_stats(char* buf, int len) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  uint64_t used = 0;
  for (const auto& kv : s.used) used = std::max(used, kv.second);
  return std::snprintf(buf, static_cast<size_t>(len),
                       "{\"limit\":%llu,\"used\":%llu,\"peak\":%llu,\"denied\":%llu,\"queuesMasked\":%llu,"
                       "\"maskBits\":%u}",
                       static_cast<unsigned long long>(s.limit), static_cast<unsigned long long>(used),
                       static_cast<unsigned long long>(s.peak.load()),
                       static_cast<unsigned long long>(s.denied.load()),
                       static_cast<unsigned long long>(s.queues_masked.load()), s.mask_bits);
}

}  // extern "C"
