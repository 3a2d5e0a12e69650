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
// The agent gives sibling slots disjoint CU ranges and refuses pools whose budgets overcommit the
// GPU (gpupool/agent/slots.py).
//
// The library is loaded into arbitrary pod images, and ROCr skips a tools library that fails to
// load — silently dropping the slot's limits. So it depends on nothing but libc (GLIBC_2.14 at
// most): no C++ standard library (fixed tables and an open-addressing hash of live allocations,
// pthread mutexes, __atomic builtins), no exceptions, RTTI or guarded statics, and the global
// state is constant-initialised (nothing runs at load or exit). Checked by
// tests/unit/test_native.py::test_share_library_needs_only_old_glibc.
#define AMD_INTERNAL_BUILD  // hsa_api_trace.h: include the sibling headers of /opt/rocm/include/hsa
#include <errno.h>
#include <fcntl.h>
#include <hsa/hsa.h>
#include <hsa/hsa_api_trace.h>
#include <hsa/hsa_ext_amd.h>
#include <pthread.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>

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

constexpr int kMaxAgents = 64;     // GPU agents one process sees (8 GPUs, or 64 CPX partitions)
constexpr int kMaxPools = 512;     // GPU-located memory pools over all of them
constexpr int kMaskWords = 128;    // CU-mask bits up to 4096

struct AgentRec {
  uint64_t handle;
  uint64_t used;      // live bytes this process holds on it
  uint32_t ordinal;   // ROCr's enumeration order
  int acct_gpu;       // account GPU index, -1 when the shared account does not cover it
};
struct PoolRec {
  uint64_t pool, agent;
};

// Live allocations (pointer or VMM handle -> agent, bytes): open addressing, linear probing,
// grown with calloc at 50 % occupancy (tombstones included). Key 0 = empty, ~0 = deleted.
struct Alloc {
  uint64_t key, agent, bytes;
};
struct AllocMap {
  Alloc* slots;
  size_t cap, live, used;  // capacity (power of two), live keys, live + tombstones
};
constexpr uint64_t kDeleted = ~0ull;

// Keys are stored +1 so that a (theoretical) VMM handle 0 is not the empty marker.
uint64_t enc(uint64_t key) { return key + 1; }

size_t slot_of(uint64_t key, size_t cap) { return static_cast<size_t>((key * 0x9E3779B97F4A7C15ull) >> 17) & (cap - 1); }

bool map_grow(AllocMap& m) {
  size_t cap = m.cap ? m.cap * 2 : 1024;
  while (m.live * 2 >= cap) cap *= 2;
  Alloc* fresh = static_cast<Alloc*>(calloc(cap, sizeof(Alloc)));
  if (!fresh) return false;
  for (size_t i = 0; i < m.cap; ++i) {
    const Alloc& a = m.slots[i];
    if (a.key == 0 || a.key == kDeleted) continue;
    size_t j = slot_of(a.key, cap);
    while (fresh[j].key) j = (j + 1) & (cap - 1);
    fresh[j] = a;
  }
  free(m.slots);
  m.slots = fresh;
  m.cap = cap;
  m.used = m.live;
  return true;
}

bool map_put(AllocMap& m, uint64_t raw, uint64_t agent, uint64_t bytes) {
  const uint64_t key = enc(raw);
  if (key == 0 || key == kDeleted) return false;
  if ((m.used + 1) * 2 > m.cap && !map_grow(m)) return false;
  size_t i = slot_of(key, m.cap), tomb = SIZE_MAX;
  for (;; i = (i + 1) & (m.cap - 1)) {
    if (m.slots[i].key == key) {
      m.slots[i].agent = agent;
      m.slots[i].bytes = bytes;
      return true;
    }
    if (m.slots[i].key == kDeleted && tomb == SIZE_MAX) tomb = i;
    if (m.slots[i].key == 0) break;
  }
  if (tomb != SIZE_MAX) i = tomb;
  else ++m.used;
  m.slots[i] = Alloc{key, agent, bytes};
  ++m.live;
  return true;
}

// Removes ``key``; true (and its record in *out) if it was there.
bool map_take(AllocMap& m, uint64_t raw, Alloc* out) {
  const uint64_t key = enc(raw);
  if (!m.cap || key == 0 || key == kDeleted) return false;
  for (size_t i = slot_of(key, m.cap);; i = (i + 1) & (m.cap - 1)) {
    if (m.slots[i].key == 0) return false;
    if (m.slots[i].key == key) {
      *out = m.slots[i];
      m.slots[i].key = kDeleted;
      --m.live;
      return true;
    }
  }
}

// A CU mask: bit words, the words in use (0 = no mask) and the bit count handed to ROCr.
struct CuMask {
  uint32_t w[kMaskWords];
  uint32_t words, bits;
};
// Per-GPU masks (GPUPOOL_CU_MASKS): a pod holding slot 0 of GPU A and slot 1 of GPU B gets each
// GPU's own slot CUs — the pod-wide union (GPUPOOL_CU_MASK) would overlap the sibling tenants'
// slots on both. Matched by the queue's agent UUID.
constexpr int kGpuMasks = 8;
struct GpuMask {
  char uuid[32];
  CuMask m;
};
constexpr int kQueueMap = 256;  // queue -> the mask it got (for the application's narrowing)
struct QueueMask {
  const hsa_queue_t* q;
  const CuMask* m;
};

struct State {
  pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;
  CoreApiTable real_core;
  AmdExtTable real_amd;
  uint64_t limit;                   // bytes per GPU; 0 = no budget
  CuMask mask;                      // the pod-wide mask (GPUPOOL_CU_MASK): GPUs without their own
  GpuMask gpu_masks[kGpuMasks];
  int n_gpu_masks;
  QueueMask qmap[kQueueMap];
  uint32_t xcds;  // XCDs of the GPU (GPUPOOL_CU_XCDS): a narrowed mask must keep a CU on each
  bool debug;
  bool pools_mapped;
  AgentRec agents[kMaxAgents];
  int n_agents;
  PoolRec pools[kMaxPools];
  int n_pools;
  AllocMap ptrs, vmem;
  uint64_t denied, queues_masked, peak, reclaimed, narrowings_refused;  // __atomic counters
  Account* acct;                    // shared account; null = per-process budget
  int32_t me;                       // pid the entries below belong to (fork changes it)
  uint64_t me_start;
  AcctEntry* mine[kAcctGpus];
};

State g_state;  // constant-initialised: no constructor at load, no destructor at exit
State& st() { return g_state; }

struct Lock {  // the state's mutex for one scope
  explicit Lock(State& s) : m(&s.mu) { pthread_mutex_lock(m); }
  ~Lock() { pthread_mutex_unlock(m); }
  Lock(const Lock&) = delete;
  Lock& operator=(const Lock&) = delete;
  pthread_mutex_t* m;
};

void count(uint64_t* c, uint64_t n = 1) { __atomic_add_fetch(c, n, __ATOMIC_RELAXED); }
uint64_t load(const uint64_t* c) { return __atomic_load_n(c, __ATOMIC_RELAXED); }

// /proc/<pid>/stat field 22 (start time in clock ticks); 0 when unreadable.
uint64_t proc_start(int32_t pid) {
  char path[64];
  snprintf(path, sizeof path, "/proc/%d/stat", pid);
  FILE* f = fopen(path, "r");
  if (!f) return 0;
  char buf[1024];
  size_t n = fread(buf, 1, sizeof buf - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* p = strrchr(buf, ')');  // comm may hold spaces: fields restart after ')'
  if (!p) return 0;
  int field = 2;
  for (++p; *p && field < 22; ++p)
    if (*p == ' ') ++field;
  return strtoull(p, nullptr, 10);
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

// This process's entry for account GPU g (claimed on first use). Caller holds s.mu.
AcctEntry* acct_entry(State& s, uint32_t g) {
  int32_t pid = static_cast<int32_t>(getpid());
  if (pid != s.me) {  // first call, or a forked child: it holds nothing of the parent's entries
    s.me = pid;
    s.me_start = proc_start(pid);
    for (AcctEntry*& e : s.mine) e = nullptr;
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
    count(&s.reclaimed, acct_reclaim(s.acct));  // table full: free the dead processes' entries
  }
  return nullptr;  // still full: charge the GPU total only
}

// Reserve ``size`` on account GPU g. Caller holds s.mu.
bool acct_charge(State& s, uint32_t g, uint64_t size) {
  uint64_t* used = &s.acct->used[g];
  bool swept = false;
  uint64_t cur = __atomic_load_n(used, __ATOMIC_ACQUIRE);
  for (;;) {
    if (cur + size > s.limit) {
      if (swept) return false;
      swept = true;  // over budget: first give back what dead processes of the pod still hold
      count(&s.reclaimed, acct_reclaim(s.acct));
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
    if (debug) fprintf(stderr, "[gpupool-share] account %s: %s\n", path, strerror(errno));
    return nullptr;
  }
  void* m = mmap(nullptr, kAcctBytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (m == MAP_FAILED) return nullptr;
  auto* a = static_cast<Account*>(m);
  if (memcmp(a->magic, kAcctMagic, sizeof kAcctMagic) != 0) {
    munmap(m, kAcctBytes);
    return nullptr;
  }
  return a;
}

// The slot's HBM limit as the agent fixed it, in a file mounted READ-ONLY into the pod
// ("GPLIMIT1 <bytes>\n"; the agent's _share_account writes it beside the account). The account
// itself must be writable — every process charges its counters there — so the limit in its header
// is the pod's to edit; this one is not. The library's budget is the smallest non-zero limit it
// is given (the env value, the account header, this file at the fixed mount path and at
// $GPUPOOL_SHARE_LIMIT): anything the pod controls can only lower it.
constexpr const char* kLimitPath = "/var/run/gpupool/share.limit";

uint64_t read_limit_file(const char* path) {
  if (!path || !*path) return 0;
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return 0;
  char buf[64] = {};
  ssize_t n = read(fd, buf, sizeof buf - 1);
  close(fd);
  if (n < 10 || memcmp(buf, "GPLIMIT1 ", 9) != 0) return 0;
  return strtoull(buf + 9, nullptr, 10);
}

void take_min(uint64_t* lim, uint64_t v) {
  if (v && (!*lim || v < *lim)) *lim = v;
}

uint64_t parse_bytes(const char* v) {
  if (!v || !*v) return 0;
  char* end = nullptr;
  double x = strtod(v, &end);
  const char* suf = end ? end : "";
  double mul = 1;
  if (!strcmp(suf, "Ki") || !strcmp(suf, "K") || !strcmp(suf, "k")) mul = 1024.0;
  else if (!strcmp(suf, "Mi") || !strcmp(suf, "M")) mul = 1024.0 * 1024;
  else if (!strcmp(suf, "Gi") || !strcmp(suf, "G")) mul = 1024.0 * 1024 * 1024;
  else if (!strcmp(suf, "Ti") || !strcmp(suf, "T")) mul = 1024.0 * 1024 * 1024 * 1024;
  return static_cast<uint64_t>(x * mul);
}

// "0-63,128-159" -> bit words (32 bits each); bits counted up to the highest set bit, rounded up
// to a multiple of 32 as hsa_amd_queue_cu_set_mask requires. Parsing stops at ';' or the end.
const char* parse_mask(CuMask& m, const char* v) {
  m.words = 0;
  m.bits = 0;
  if (!v || !*v) return v;
  const char* p = v;
  while (*p && *p != ';') {
    char* end = nullptr;
    long lo = strtol(p, &end, 10);
    bool ok = end != p;
    long hi = lo;
    p = end;
    if (ok && *p == '-') {
      const char* q = p + 1;
      hi = strtol(q, &end, 10);
      ok = end != q;
      p = end;
    }
    while (*p && *p != ',' && *p != ';') ++p;  // skip to the next range (malformed tails are ignored)
    if (*p == ',') ++p;
    if (!ok || lo < 0 || hi < lo || hi >= kMaskWords * 32) continue;
    for (long b = lo; b <= hi; ++b) {
      const uint32_t w = static_cast<uint32_t>(b) / 32;
      m.w[w] |= 1u << (b % 32);
      if (w + 1 > m.words) m.words = w + 1;
    }
  }
  m.bits = m.words * 32;
  return p;
}

// "GPU-aaaa=0-63,128-159;GPU-bbbb=64-127" -> s.gpu_masks
void parse_gpu_masks(State& s, const char* v) {
  s.n_gpu_masks = 0;
  const char* p = v;
  while (p && *p && s.n_gpu_masks < kGpuMasks) {
    const char* eq = strchr(p, '=');
    if (!eq) break;
    GpuMask& g = s.gpu_masks[s.n_gpu_masks];
    size_t n = static_cast<size_t>(eq - p);
    if (n == 0 || n >= sizeof g.uuid) break;
    memcpy(g.uuid, p, n);
    g.uuid[n] = 0;
    p = parse_mask(g.m, eq + 1);
    if (g.m.words) ++s.n_gpu_masks;
    if (p && *p == ';') ++p;
  }
}

// The mask a queue on ``agent`` gets: its GPU's own (by UUID), else the pod-wide one, else none.
const CuMask* mask_for(State& s, hsa_agent_t agent) {
  if (s.n_gpu_masks) {
    char uuid[64] = {};
    if (s.real_core.hsa_agent_get_info_fn(agent, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_UUID), uuid) ==
        HSA_STATUS_SUCCESS) {
      uuid[sizeof uuid - 1] = 0;
      for (int i = 0; i < s.n_gpu_masks; ++i)
        if (strcmp(s.gpu_masks[i].uuid, uuid) == 0) return &s.gpu_masks[i].m;
    }
  }
  return s.mask.words ? &s.mask : nullptr;
}

AgentRec* agent_rec(State& s, uint64_t handle) {
  for (int i = 0; i < s.n_agents; ++i)
    if (s.agents[i].handle == handle) return &s.agents[i];
  return nullptr;
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
  const uint32_t n = s.acct->ngpus < static_cast<uint32_t>(kAcctGpus) ? s.acct->ngpus : kAcctGpus;
  for (uint32_t g = 0; g < n; ++g) {
    const char* id = table + g * kAcctUuidBytes;
    if (id[0] && strlen(uuid) < kAcctUuidBytes && strncmp(id, uuid, kAcctUuidBytes) == 0) return static_cast<int>(g);
  }
  if (s.debug) fprintf(stderr, "[gpupool-share] GPU %s is not in the pod's account\n", uuid);
  return -1;
}

hsa_status_t collect_pool(hsa_amd_memory_pool_t pool, void* agent_handle) {
  State& s = st();
  hsa_amd_memory_pool_location_t loc{};
  if (s.real_amd.hsa_amd_memory_pool_get_info_fn &&
      s.real_amd.hsa_amd_memory_pool_get_info_fn(pool, HSA_AMD_MEMORY_POOL_INFO_LOCATION, &loc) == HSA_STATUS_SUCCESS &&
      loc == HSA_AMD_MEMORY_POOL_LOCATION_GPU && s.n_pools < kMaxPools)
    s.pools[s.n_pools++] = PoolRec{pool.handle, *static_cast<uint64_t*>(agent_handle)};
  return HSA_STATUS_SUCCESS;
}

hsa_status_t collect_agent(hsa_agent_t agent, void*) {
  State& s = st();
  hsa_device_type_t type{};
  if (s.real_core.hsa_agent_get_info_fn(agent, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS ||
      type != HSA_DEVICE_TYPE_GPU || s.n_agents >= kMaxAgents)
    return HSA_STATUS_SUCCESS;
  AgentRec& r = s.agents[s.n_agents];
  r.handle = agent.handle;
  r.used = 0;
  r.ordinal = static_cast<uint32_t>(s.n_agents);  // ROCr's enumeration order
  r.acct_gpu = s.acct ? acct_index(s, agent, r.ordinal) : -1;
  ++s.n_agents;
  uint64_t h = agent.handle;
  if (s.real_amd.hsa_amd_agent_iterate_memory_pools_fn)
    s.real_amd.hsa_amd_agent_iterate_memory_pools_fn(agent, collect_pool, &h);
  return HSA_STATUS_SUCCESS;
}

void map_agents(State& s) {  // caller holds s.mu
  if (s.pools_mapped) return;
  s.pools_mapped = true;
  if (s.real_core.hsa_iterate_agents_fn) s.real_core.hsa_iterate_agents_fn(collect_agent, nullptr);
}

// pool -> its GPU agent's record (null if the pool is not GPU memory). Caller holds s.mu.
AgentRec* agent_of(hsa_amd_memory_pool_t pool) {
  State& s = st();
  map_agents(s);
  for (int i = 0; i < s.n_pools; ++i)
    if (s.pools[i].pool == pool.handle) return agent_rec(s, s.pools[i].agent);
  return nullptr;
}

// The account slot of an agent: its account GPU when the shared account covers it, else -1.
int shared_index(const State& s, const AgentRec* a) { return s.acct && a ? a->acct_gpu : -1; }

// Live bytes against the budget on ``a``: the pod's total when shared. Caller holds s.mu.
uint64_t budget_used(State& s, const AgentRec* a) {
  int g = shared_index(s, a);
  if (g >= 0) return __atomic_load_n(&s.acct->used[g], __ATOMIC_ACQUIRE);
  return a ? a->used : 0;
}

// Reserve ``size`` bytes on ``a``; false when over budget. Caller holds s.mu.
bool charge(AgentRec* a, uint64_t size) {
  State& s = st();
  int g = shared_index(s, a);
  bool ok = g >= 0 ? acct_charge(s, static_cast<uint32_t>(g), size) : !(s.limit && a->used + size > s.limit);
  if (!ok) {
    count(&s.denied);
    if (s.debug)
      fprintf(stderr, "[gpupool-share] deny %llu B: %llu in use of %llu%s\n", static_cast<unsigned long long>(size),
              static_cast<unsigned long long>(budget_used(s, a)), static_cast<unsigned long long>(s.limit),
              g >= 0 ? " (pod total)" : "");
    return false;
  }
  a->used += size;
  uint64_t pk = __atomic_load_n(&s.peak, __ATOMIC_RELAXED);
  while (a->used > pk && !__atomic_compare_exchange_n(&s.peak, &pk, a->used, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {}
  return true;
}

// Return ``size`` bytes on ``a``. Caller holds s.mu.
void uncharge(AgentRec* a, uint64_t size) {
  State& s = st();
  if (!a) return;
  a->used = a->used > size ? a->used - size : 0;
  int g = shared_index(s, a);
  if (g >= 0) acct_release(s, static_cast<uint32_t>(g), size);
}

hsa_status_t w_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t flags, void** ptr) {
  State& s = st();
  AgentRec* a = nullptr;
  {
    Lock g(s);
    a = agent_of(pool);
    if (a && !charge(a, size)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  hsa_status_t r = s.real_amd.hsa_amd_memory_pool_allocate_fn(pool, size, flags, ptr);
  Lock g(s);
  if (!a) return r;
  if (r == HSA_STATUS_SUCCESS && ptr && *ptr) {
    if (!map_put(s.ptrs, reinterpret_cast<uint64_t>(*ptr), a->handle, size)) uncharge(a, size);  // OOM: untracked
  } else {
    uncharge(a, size);
  }
  return r;
}

hsa_status_t w_pool_free(void* ptr) {
  State& s = st();
  {
    Lock g(s);
    Alloc rec;
    if (map_take(s.ptrs, reinterpret_cast<uint64_t>(ptr), &rec)) uncharge(agent_rec(s, rec.agent), rec.bytes);
  }
  return s.real_amd.hsa_amd_memory_pool_free_fn(ptr);
}

hsa_status_t w_vmem_create(hsa_amd_memory_pool_t pool, size_t size, hsa_amd_memory_type_t type, uint64_t flags,
                           hsa_amd_vmem_alloc_handle_t* handle) {
  State& s = st();
  AgentRec* a = nullptr;
  {
    Lock g(s);
    a = agent_of(pool);
    if (a && !charge(a, size)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  hsa_status_t r = s.real_amd.hsa_amd_vmem_handle_create_fn(pool, size, type, flags, handle);
  Lock g(s);
  if (!a) return r;
  if (r == HSA_STATUS_SUCCESS && handle) {
    if (!map_put(s.vmem, handle->handle, a->handle, size)) uncharge(a, size);
  } else {
    uncharge(a, size);
  }
  return r;
}

hsa_status_t w_vmem_release(hsa_amd_vmem_alloc_handle_t handle) {
  State& s = st();
  {
    Lock g(s);
    Alloc rec;
    if (map_take(s.vmem, handle.handle, &rec)) uncharge(agent_rec(s, rec.agent), rec.bytes);
  }
  return s.real_amd.hsa_amd_vmem_handle_release_fn(handle);
}

hsa_status_t w_pool_get_info(hsa_amd_memory_pool_t pool, hsa_amd_memory_pool_info_t attr, void* value) {
  State& s = st();
  hsa_status_t r = s.real_amd.hsa_amd_memory_pool_get_info_fn(pool, attr, value);
  if (r != HSA_STATUS_SUCCESS || attr != HSA_AMD_MEMORY_POOL_INFO_SIZE || !s.limit || !value) return r;
  Lock g(s);
  if (agent_of(pool)) {
    size_t* sz = static_cast<size_t*>(value);
    if (*sz > s.limit) *sz = static_cast<size_t>(s.limit);
  }
  return r;
}

hsa_status_t w_agent_get_info(hsa_agent_t agent, hsa_agent_info_t attr, void* value) {
  State& s = st();
  hsa_status_t r = s.real_core.hsa_agent_get_info_fn(agent, attr, value);
  if (r != HSA_STATUS_SUCCESS || !s.limit || !value ||
      static_cast<int>(attr) != static_cast<int>(HSA_AMD_AGENT_INFO_MEMORY_AVAIL))
    return r;
  Lock g(s);
  map_agents(s);
  if (AgentRec* a = agent_rec(s, agent.handle)) {
    uint64_t* avail = static_cast<uint64_t*>(value);
    uint64_t u = budget_used(s, a);  // with a shared account: what the whole pod holds
    uint64_t left = s.limit > u ? s.limit - u : 0;
    if (*avail > left) *avail = left;
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
  if (r != HSA_STATUS_SUCCESS || !queue || !*queue || !is_gpu(agent)) return r;
  const CuMask* cm = mask_for(s, agent);
  if (!cm) return r;
  {
    Lock g(s);  // remember the queue's mask: the application may narrow it later
    int free_at = -1;
    for (int i = 0; i < kQueueMap; ++i) {
      if (s.qmap[i].q == *queue) {
        free_at = i;
        break;
      }
      if (free_at < 0 && !s.qmap[i].q) free_at = i;
    }
    if (free_at >= 0) s.qmap[free_at] = QueueMask{*queue, cm};
  }
  hsa_status_t m = s.real_amd.hsa_amd_queue_cu_set_mask_fn(*queue, cm->bits, cm->w);
  if (m == HSA_STATUS_SUCCESS || static_cast<int>(m) == static_cast<int>(HSA_STATUS_CU_MASK_REDUCED))
    count(&s.queues_masked);
  if (s.debug)
    fprintf(stderr, "[gpupool-share] queue %p CU mask (%u bits): status %d\n", static_cast<void*>(*queue), cm->bits,
            static_cast<int>(m));
  return r;
}

// The mask a queue got at creation. A queue the map does not hold (created before the library
// was loaded, or beyond kQueueMap live queues): with per-GPU masks the union is NOT a safe stand-in
// — it overlaps the sibling tenants' slots on every GPU — so *unknown is set and the caller keeps
// whatever the queue has; with one pod-wide mask that mask is the queue's.
const CuMask* queue_mask(State& s, const hsa_queue_t* q, bool* unknown) {
  Lock g(s);
  *unknown = false;
  for (int i = 0; i < kQueueMap; ++i)
    if (s.qmap[i].q == q) return s.qmap[i].m;
  if (s.n_gpu_masks) {
    *unknown = true;
    return nullptr;
  }
  return s.mask.words ? &s.mask : nullptr;
}

// Queues go away: their map entries are freed, so a process that creates and destroys queues all
// its life (a stream per request) never runs out of entries.
hsa_status_t w_queue_destroy(hsa_queue_t* queue) {
  State& s = st();
  {
    Lock g(s);
    for (int i = 0; i < kQueueMap; ++i)
      if (s.qmap[i].q == queue) s.qmap[i] = QueueMask{};
  }
  return s.real_core.hsa_queue_destroy_fn(queue);
}

// Does ``m`` leave at least one CU on every XCD? CU-mask bit b lands on XCD b % xcds (ROCr
// interleaves CUs over the XCDs), and a mask that leaves any XCD without CUs is silently NOT
// applied by the driver (measured, profiles/r4b_cu_mask_layouts.txt): the queue would then run
// on all 256 CUs, its slot neighbours' included.
bool covers_every_xcd(const State& s, const uint32_t* m, uint32_t words) {
  if (s.xcds <= 1) return true;
  uint32_t seen = 0;  // one bit per XCD (at most 32)
  const uint32_t want = s.xcds >= 32 ? ~0u : (1u << s.xcds) - 1;
  for (uint32_t w = 0; w < words && seen != want; ++w)
    for (uint32_t b = 0; b < 32 && m[w] >> b; ++b)
      if (m[w] >> b & 1u) seen |= 1u << ((w * 32 + b) % s.xcds % 32);
  return (seen & want) == want;
}

hsa_status_t w_queue_cu_set_mask(const hsa_queue_t* queue, uint32_t bits, const uint32_t* mask) {
  // the application's own mask (hipExtStreamCreateWithCUMask) can only narrow the slot's
  State& s = st();
  bool unknown = false;
  const CuMask* cm = queue_mask(s, queue, &unknown);
  if (unknown) {  // not ours to widen or narrow blind: the queue keeps its creation mask
    count(&s.narrowings_refused);
    return HSA_STATUS_SUCCESS;
  }
  if (!cm) return s.real_amd.hsa_amd_queue_cu_set_mask_fn(queue, bits, mask);
  uint32_t m[kMaskWords];
  bool any = false;
  for (uint32_t i = 0; i < cm->words; ++i) {
    m[i] = cm->w[i];
    if (bits > 0 && mask) m[i] &= i < bits / 32 ? mask[i] : 0u;
    any = any || m[i];
  }
  // nothing left, or a narrowing that empties an XCD (the driver would then drop the mask and run
  // the queue on every CU): the slot's own mask
  if (bits > 0 && mask && (!any || !covers_every_xcd(s, m, cm->words))) {
    for (uint32_t i = 0; i < cm->words; ++i) m[i] = cm->w[i];
    count(&s.narrowings_refused);
  }
  return s.real_amd.hsa_amd_queue_cu_set_mask_fn(queue, cm->bits, m);
}

}  // namespace

extern "C" {

// ROCr tools-library entry point (HSA_TOOLS_LIB): install the wrappers into the dispatch table.
__attribute__((visibility("default"))) bool OnLoad(HsaApiTable* table, uint64_t runtime_version,
                                                   uint64_t failed_tool_count, const char* const* failed_tool_names) {
  if (!table || !table->core_ || !table->amd_ext_) return false;
  State& s = st();
  Lock g(s);
  s.real_core = *table->core_;
  s.real_amd = *table->amd_ext_;
  parse_mask(s.mask, getenv("GPUPOOL_CU_MASK"));
  parse_gpu_masks(s, getenv("GPUPOOL_CU_MASKS"));
  const char* xcds = getenv("GPUPOOL_CU_XCDS");
  s.xcds = xcds && *xcds ? static_cast<uint32_t>(strtoul(xcds, nullptr, 10)) : 0;
  const char* dbg = getenv("GPUPOOL_SHARE_DEBUG");
  s.debug = dbg && *dbg && *dbg != '0';
  s.acct = acct_open(getenv("GPUPOOL_SHARE_ACCOUNT"), s.debug);
  uint64_t lim = 0;
  take_min(&lim, parse_bytes(getenv("GPUPOOL_HBM_LIMIT_BYTES")));
  if (s.acct) take_min(&lim, s.acct->limit);
  take_min(&lim, read_limit_file(kLimitPath));
  take_min(&lim, read_limit_file(getenv("GPUPOOL_SHARE_LIMIT")));
  s.limit = lim;
  if (s.limit) {
    table->amd_ext_->hsa_amd_memory_pool_allocate_fn = w_pool_allocate;
    table->amd_ext_->hsa_amd_memory_pool_free_fn = w_pool_free;
    table->amd_ext_->hsa_amd_vmem_handle_create_fn = w_vmem_create;
    table->amd_ext_->hsa_amd_vmem_handle_release_fn = w_vmem_release;
    table->amd_ext_->hsa_amd_memory_pool_get_info_fn = w_pool_get_info;
    table->core_->hsa_agent_get_info_fn = w_agent_get_info;
  }
  if (s.mask.words || s.n_gpu_masks) {
    table->core_->hsa_queue_create_fn = w_queue_create;
    table->core_->hsa_queue_destroy_fn = w_queue_destroy;
    table->amd_ext_->hsa_amd_queue_cu_set_mask_fn = w_queue_cu_set_mask;
  }
  if (s.debug)
    fprintf(stderr, "[gpupool-share] loaded: HBM limit %llu B per GPU (%s), CU mask %u bits\n",
            static_cast<unsigned long long>(s.limit), s.acct ? "pod total" : "per process", s.mask.bits);
  return true;
}

__attribute__((visibility("default"))) void OnUnload() {}

// Counters for tests and diagnostics: JSON into buf.
__attribute__((visibility("default"))) int gpupool_share_stats(char* buf, int len) {
  State& s = st();
  Lock g(s);
  uint64_t used = 0, shared = 0;
  for (int i = 0; i < s.n_agents; ++i) {
    const AgentRec* a = &s.agents[i];
    if (a->used > used) used = a->used;
    if (shared_index(s, a) >= 0) {
      uint64_t u = budget_used(s, a);
      if (u > shared) shared = u;
    }
  }
  return snprintf(buf, static_cast<size_t>(len),
                  "{\"limit\":%llu,\"used\":%llu,\"peak\":%llu,\"denied\":%llu,\"queuesMasked\":%llu,"
                  "\"maskBits\":%u,\"shared\":%d,\"podUsed\":%llu,\"reclaimed\":%llu,"
                  "\"narrowingsRefused\":%llu}",
                  static_cast<unsigned long long>(s.limit), static_cast<unsigned long long>(used),
                  static_cast<unsigned long long>(load(&s.peak)), static_cast<unsigned long long>(load(&s.denied)),
                  static_cast<unsigned long long>(load(&s.queues_masked)), s.mask.bits, s.acct ? 1 : 0,
                  static_cast<unsigned long long>(shared), static_cast<unsigned long long>(load(&s.reclaimed)),
                  static_cast<unsigned long long>(load(&s.narrowings_refused)));
}

}  // extern "C"
