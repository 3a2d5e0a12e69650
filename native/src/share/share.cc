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
//     pod's live VRAM on that GPU would exceed the budget (HIP reports hipErrorOutOfMemory);
//     hsa_amd_memory_pool_free / hsa_amd_vmem_handle_release return the bytes. The pool SIZE and
//     the agent's MEMORY_AVAIL report the budget, so hipMemGetInfo / torch.cuda.mem_get_info and
//     the caching allocators that size themselves from it see the slot, not the whole GPU.
//   * CU share (GPUPOOL_CU_MASK, CU-mask bit ranges like "0-63" or "0-31,128-159"): every HSA
//     queue created on a GPU gets hsa_amd_queue_cu_set_mask(mask), and an application's own
//     hipExtStreamCreateWithCUMask mask is intersected with it — waves of this process can only
//     be dispatched to the slot's CUs.
//
// The budget covers every process of the container: the agent creates one account file per
// allocation (GPUPOOL_SHARE_ACCOUNT, mounted into the container) and every process charges its
// VRAM there with atomic compare-and-swap on the shared page, so a pod running 4 ranks or a
// DataLoader's worker processes on its slot still gets (slots x hbmBytesPerSlot) in total, not
// per process. Each process also records what it holds in its own entry (pid + start time), and
// a process that finds the budget exhausted first returns the bytes of entries whose process is
// gone (killed by OOM, SIGKILL — no free ever ran). Without the file the budget is per process.
// The agent gives sibling slots disjoint CU ranges and budgets that sum to at most the GPU's HBM.
#define AMD_INTERNAL_BUILD  // hsa_api_trace.h: include the sibling headers of /opt/rocm/include/hsa
#include <fcntl.h>
#include <hsa/hsa.h>
#include <hsa/hsa_api_trace.h>
#include <hsa/hsa_ext_amd.h>
#include <signal.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
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

// ---- the shared account file (written by the agent, gpupool/agent/agent.py _share_account) ----
// [0,64) header, [64,128) live bytes per account GPU, [128,8192) per-process entries,
// version 2: [8192,8448) the account GPUs' identities — 8 NUL-padded 32-byte strings, the
// HSA_AMD_AGENT_INFO_UUID ("GPU-<hex>", amdsmi's hip_uuid) of account GPU g at 8192 + 32 g —
// then the allocation's slot ids as text (the agent's bookkeeping; ignored here). Version 1 files
// have no identities: account GPU g is the process's g-th GPU agent.
constexpr size_t kAcctBytes = 16384;
constexpr int kAcctGpus = 8;
constexpr int kAcctEntries = (8192 - 128) / 32;
constexpr size_t kAcctUuidsAt = 8192, kAcctUuidBytes = 32;
constexpr char kAcctMagic[8] = {'G', 'P', 'S', 'H', 'A', 'R', 'E', '1'};

struct AcctEntry {
  int32_t pid;     // 0 free, -1 being claimed or reclaimed, else the owning process
  uint32_t gpu;    // account GPU index (see the layout above)
  uint64_t start;  // the owner's start time (/proc/<pid>/stat field 22): pid reuse is not a match
  uint64_t bytes;  // live bytes the owner holds on ``gpu``
  uint64_t pad;
};
struct Account {
  char magic[8];
  uint64_t limit;  // bytes per GPU (the agent writes GPUPOOL_HBM_LIMIT_BYTES here too)
  uint32_t version, ngpus;
  uint64_t pad[5];
  uint64_t used[kAcctGpus];
  AcctEntry entries[kAcctEntries];
};
static_assert(sizeof(Account) == 8192, "account layout");

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
  std::map<uint64_t, uint64_t> used;        // agent handle -> live bytes (this process)
  std::map<uint64_t, uint32_t> ordinal;     // agent handle -> ROCr's enumeration order
  std::map<uint64_t, int> acct_gpu;         // agent handle -> account GPU index (-1: not in the account)
  std::unordered_map<void*, std::pair<uint64_t, uint64_t>> ptrs;       // ptr -> (agent, bytes)
  std::unordered_map<uint64_t, std::pair<uint64_t, uint64_t>> vmem;    // handle -> (agent, bytes)
  std::atomic<uint64_t> denied{0}, queues_masked{0}, peak{0}, reclaimed{0};
  Account* acct = nullptr;                  // shared account; null = per-process budget
  int32_t me = 0;                           // pid the entries below belong to (fork changes it)
  uint64_t me_start = 0;
  AcctEntry* mine[kAcctGpus] = {};
};

State& st() {
  static State* s = new State();  // never destroyed: HSA may call in during process exit
  return *s;
}

// /proc/<pid>/stat field 22 (start time in clock ticks); 0 when unreadable.
uint64_t proc_start(int32_t pid) {
  char path[64];
  std::snprintf(path, sizeof path, "/proc/%d/stat", pid);
  FILE* f = std::fopen(path, "r");
  if (!f) return 0;
  char buf[1024];
  size_t n = std::fread(buf, 1, sizeof buf - 1, f);
  std::fclose(f);
  buf[n] = 0;
  const char* p = std::strrchr(buf, ')');  // comm may hold spaces: fields restart after ')'
  if (!p) return 0;
  int field = 2;
  for (++p; *p && field < 22; ++p)
    if (*p == ' ') ++field;
  return std::strtoull(p, nullptr, 10);
}

bool proc_alive(int32_t pid, uint64_t start) {
  if (kill(pid, 0) != 0 && errno == ESRCH) return false;
  uint64_t now = proc_start(pid);
  return now == 0 || start == 0 || now == start;  // unreadable: assume alive (never over-return)
}

void sat_sub(uint64_t* v, uint64_t n) {
  uint64_t cur = __atomic_load_n(v, __ATOMIC_ACQUIRE);
  while (!__atomic_compare_exchange_n(v, &cur, cur > n ? cur - n : 0, true, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {}
}

// Return the bytes of entries whose process is gone. Returns the bytes reclaimed.
uint64_t acct_reclaim(Account* a) {
  uint64_t total = 0;
  for (AcctEntry& e : a->entries) {
    int32_t pid = __atomic_load_n(&e.pid, __ATOMIC_ACQUIRE);
    if (pid <= 0 || proc_alive(pid, __atomic_load_n(&e.start, __ATOMIC_ACQUIRE))) continue;
    if (!__atomic_compare_exchange_n(&e.pid, &pid, -1, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE))
      continue;  // another process is reclaiming it
    uint64_t b = __atomic_exchange_n(&e.bytes, 0, __ATOMIC_ACQ_REL);
    if (e.gpu < kAcctGpus) sat_sub(&a->used[e.gpu], b);
    total += b;
    __atomic_store_n(&e.pid, 0, __ATOMIC_RELEASE);
  }
  return total;
}

// This process's entry for GPU ordinal g (claimed on first use). Caller holds s.mu.
AcctEntry* acct_entry(State& s, uint32_t g) {
  int32_t pid = static_cast<int32_t>(getpid());
  if (pid != s.me) {  // first call, or a forked child: it holds nothing of the parent's entries
    s.me = pid;
    s.me_start = proc_start(pid);
    std::fill(std::begin(s.mine), std::end(s.mine), nullptr);
  }
  if (s.mine[g]) return s.mine[g];
  for (int pass = 0; pass < 2; ++pass) {
    for (AcctEntry& e : s.acct->entries) {
      int32_t free_pid = 0;
      if (!__atomic_compare_exchange_n(&e.pid, &free_pid, -1, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE))
        continue;
      e.gpu = g;
      __atomic_store_n(&e.start, s.me_start, __ATOMIC_RELEASE);
      __atomic_store_n(&e.bytes, 0, __ATOMIC_RELEASE);
      __atomic_store_n(&e.pid, pid, __ATOMIC_RELEASE);
      return s.mine[g] = &e;
    }
    s.reclaimed.fetch_add(acct_reclaim(s.acct));  // table full: free the dead processes' entries
  }
  return nullptr;  // still full: charge the GPU total only
}

// Reserve ``size`` on GPU ordinal g in the shared account. Caller holds s.mu.
bool acct_charge(State& s, uint32_t g, uint64_t size) {
  uint64_t* used = &s.acct->used[g];
  bool swept = false;
  uint64_t cur = __atomic_load_n(used, __ATOMIC_ACQUIRE);
  for (;;) {
    if (cur + size > s.limit) {
      if (swept) return false;
      swept = true;  // over budget: first give back what dead processes of the pod still hold
      s.reclaimed.fetch_add(acct_reclaim(s.acct));
      cur = __atomic_load_n(used, __ATOMIC_ACQUIRE);
      continue;
    }
    if (__atomic_compare_exchange_n(used, &cur, cur + size, true, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) break;
  }
  // total first, own entry second: a crash in between leaks ``size`` until the file is replaced
  // but never lets a reclaim return bytes the total does not hold
  if (AcctEntry* e = acct_entry(s, g)) __atomic_add_fetch(&e->bytes, size, __ATOMIC_ACQ_REL);
  return true;
}

void acct_release(State& s, uint32_t g, uint64_t size) {
  if (AcctEntry* e = acct_entry(s, g)) sat_sub(&e->bytes, size);
  sat_sub(&s.acct->used[g], size);
}

Account* acct_open(const char* path, bool debug) {
  if (!path || !*path) return nullptr;
  int fd = open(path, O_RDWR | O_CLOEXEC);
  if (fd < 0) {
    if (debug) std::fprintf(stderr, "[gpupool-share] account %s: %s\n", path, std::strerror(errno));
    return nullptr;
  }
  void* m = mmap(nullptr, kAcctBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return nullptr;
  auto* a = static_cast<Account*>(m);
  if (std::memcmp(a->magic, kAcctMagic, sizeof kAcctMagic) != 0) {
    munmap(m, kAcctBytes);
    return nullptr;
  }
  return a;
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

// The account GPU of a GPU agent. Version 2 accounts name their GPUs, so every process of the pod
// charges the same counter for the same physical GPU whatever subset of GPUs it sees (a launcher's
// per-rank ROCR_VISIBLE_DEVICES reorders and narrows the enumeration); a GPU the account does not
// name is not budgeted through it (-1). Version 1: the agent's ordinal. Caller holds s.mu.
int acct_index(State& s, hsa_agent_t agent, uint32_t ordinal) {
  if (s.acct->version < 2) return ordinal < static_cast<uint32_t>(kAcctGpus) ? static_cast<int>(ordinal) : -1;
  char uuid[64] = {};
  if (s.real_core.hsa_agent_get_info_fn(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_UUID), uuid) !=
      HSA_STATUS_SUCCESS)
    return -1;
  uuid[sizeof uuid - 1] = 0;
  const char* table = reinterpret_cast<const char*>(s.acct) + kAcctUuidsAt;
  const uint32_t n = std::min<uint32_t>(s.acct->ngpus, kAcctGpus);
  for (uint32_t g = 0; g < n; ++g) {
    const char* id = table + g * kAcctUuidBytes;
    if (id[0] && std::strncmp(id, uuid, kAcctUuidBytes) == 0 && std::strlen(uuid) < kAcctUuidBytes)
      return static_cast<int>(g);
  }
  if (s.debug) std::fprintf(stderr, "[gpupool-share] GPU %s is not in the pod's account\n", uuid);
  return -1;
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
  const uint32_t ord = static_cast<uint32_t>(s.ordinal.size());  // ROCr's enumeration order
  s.ordinal.emplace(h, ord);
  if (s.acct) s.acct_gpu.emplace(h, acct_index(s, agent, ord));
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
// The account slot of ``agent``: its ordinal when the shared account covers it, else -1.
int shared_index(State& s, uint64_t agent) {
  if (!s.acct) return -1;
  auto it = s.acct_gpu.find(agent);
  return it != s.acct_gpu.end() ? it->second : -1;
}

// Live bytes against the budget on ``agent``: the pod's total when shared. Caller holds s.mu.
uint64_t budget_used(State& s, uint64_t agent) {
  int g = shared_index(s, agent);
  if (g >= 0) return __atomic_load_n(&s.acct->used[g], __ATOMIC_ACQUIRE);
  auto it = s.used.find(agent);
  return it == s.used.end() ? 0 : it->second;
}

bool charge(uint64_t agent, size_t size) {
  State& s = st();
  uint64_t& u = s.used[agent];
  int g = shared_index(s, agent);
  bool ok = g >= 0 ? acct_charge(s, static_cast<uint32_t>(g), size) : !(s.limit && u + size > s.limit);
  if (!ok) {
    s.denied.fetch_add(1);
    if (s.debug)
      std::fprintf(stderr, "[gpupool-share] deny %zu B: %llu in use of %llu%s\n", size,
                   static_cast<unsigned long long>(budget_used(s, agent)),
                   static_cast<unsigned long long>(s.limit), g >= 0 ? " (pod total)" : "");
    return false;
  }
  u += size;
  uint64_t pk = s.peak.load();
  while (u > pk && !s.peak.compare_exchange_weak(pk, u)) {}
  return true;
}

// Return ``size`` bytes on ``agent``. Caller holds s.mu.
void uncharge(uint64_t agent, uint64_t size) {
  State& s = st();
  uint64_t& u = s.used[agent];
  u = u > size ? u - size : 0;
  int g = shared_index(s, agent);
  if (g >= 0) acct_release(s, static_cast<uint32_t>(g), size);
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
  else uncharge(agent, size);
  return r;
}

hsa_status_t w_pool_free(void* ptr) {
  State& s = st();
  {
    std::lock_guard<std::mutex> g(s.mu);
    auto it = s.ptrs.find(ptr);
    if (it != s.ptrs.end()) {
      uncharge(it->second.first, it->second.second);
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
  else uncharge(agent, size);
  return r;
}

hsa_status_t w_vmem_release(hsa_amd_vmem_alloc_handle_t handle) {
  State& s = st();
  {
    std::lock_guard<std::mutex> g(s.mu);
    auto it = s.vmem.find(handle.handle);
    if (it != s.vmem.end()) {
      uncharge(it->second.first, it->second.second);
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
  if (s.used.count(agent.handle)) {
    uint64_t* avail = static_cast<uint64_t*>(value);
    uint64_t u = budget_used(s, agent.handle);  // with a shared account: what the whole pod holds
    uint64_t left = s.limit > u ? s.limit - u : 0;
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
  s.acct = acct_open(std::getenv("GPUPOOL_SHARE_ACCOUNT"), s.debug);
  if (s.acct && s.acct->limit) s.limit = s.acct->limit;  // the agent's number wins
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
    std::fprintf(stderr, "[gpupool-share] loaded: HBM limit %llu B per GPU (%s), CU mask %u bits\n",
                 static_cast<unsigned long long>(s.limit), s.acct ? "pod total" : "per process", s.mask_bits);
  return true;
}

__attribute__((visibility("default"))) void OnUnload() {}

// Counters for tests and diagnostics: JSON into buf.
__attribute__((visibility("default"))) int gpupool_share_stats(char* buf, int len) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  uint64_t used = 0, shared = 0;
  for (const auto& kv : s.used) {
    used = std::max(used, kv.second);
    if (shared_index(s, kv.first) >= 0) shared = std::max(shared, budget_used(s, kv.first));
  }
  return std::snprintf(buf, static_cast<size_t>(len),
                       "{\"limit\":%llu,\"used\":%llu,\"peak\":%llu,\"denied\":%llu,\"queuesMasked\":%llu,"
                       "\"maskBits\":%u,\"shared\":%d,\"podUsed\":%llu,\"reclaimed\":%llu}",
                       static_cast<unsigned long long>(s.limit), static_cast<unsigned long long>(used),
                       static_cast<unsigned long long>(s.peak.load()),
                       static_cast<unsigned long long>(s.denied.load()),
                       static_cast<unsigned long long>(s.queues_masked.load()), s.mask_bits, s.acct ? 1 : 0,
                       static_cast<unsigned long long>(shared), static_cast<unsigned long long>(s.reclaimed.load()));
}

}  // extern "C"
