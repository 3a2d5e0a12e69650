// libgpupool_share.so on the CPU: OnLoad() against a fake HSA dispatch table (one GPU agent with a
// VRAM pool, one CPU agent with a system pool), then the wrapped entry points: HBM budget per GPU,
// frees returning budget, VMM handles counted, pool SIZE / MEMORY_AVAIL reporting the slot, CU
// masks on new GPU queues and intersected with the application's own.
#define AMD_INTERNAL_BUILD
#include <dlfcn.h>
#include <fcntl.h>
#include <hsa/hsa.h>
#include <hsa/hsa_api_trace.h>
#include <hsa/hsa_ext_amd.h>
#include <sys/wait.h>
#include <unistd.h>

#include <climits>
#include <cstring>
#include <cstdlib>
#include <string>
#include <vector>

#include "testing.h"

namespace {

constexpr uint64_t kGpu = 0x1000, kCpu = 0x2000, kGpu2 = 0x3000, kGpuPool = 0x10, kCpuPool = 0x20, kGpuPool2 = 0x30;
constexpr size_t kMi = 1024 * 1024;
uint64_t g_next_ptr = 0x7000000;
std::vector<uint32_t> g_last_mask;
uint32_t g_last_bits = 0;
int g_masks_set = 0;
std::vector<uint64_t> g_gpus = {kGpu};  // the GPU agents this "process" sees, in ROCr's order

const char* uuid_of(uint64_t agent) { return agent == kGpu ? "GPU-aaaa000000000001" : "GPU-bbbb000000000002"; }

hsa_status_t f_iterate_agents(hsa_status_t (*cb)(hsa_agent_t, void*), void* data) {
  cb(hsa_agent_t{kCpu}, data);
  for (uint64_t g : g_gpus) cb(hsa_agent_t{g}, data);
  return HSA_STATUS_SUCCESS;
}
hsa_status_t f_agent_get_info(hsa_agent_t a, hsa_agent_info_t attr, void* v) {
  if (attr == HSA_AGENT_INFO_DEVICE) {
    *static_cast<hsa_device_type_t*>(v) = a.handle != kCpu ? HSA_DEVICE_TYPE_GPU : HSA_DEVICE_TYPE_CPU;
    return HSA_STATUS_SUCCESS;
  }
  if (static_cast<int>(attr) == static_cast<int>(HSA_AMD_AGENT_INFO_UUID)) {
    std::strcpy(static_cast<char*>(v), a.handle == kCpu ? "CPU-XX" : uuid_of(a.handle));
    return HSA_STATUS_SUCCESS;
  }
  if (static_cast<int>(attr) == static_cast<int>(HSA_AMD_AGENT_INFO_MEMORY_AVAIL)) {
    *static_cast<uint64_t*>(v) = 288ull << 30;
    return HSA_STATUS_SUCCESS;
  }
  return HSA_STATUS_ERROR_INVALID_ARGUMENT;
}
hsa_status_t f_iterate_pools(hsa_agent_t a, hsa_status_t (*cb)(hsa_amd_memory_pool_t, void*), void* data) {
  cb(hsa_amd_memory_pool_t{a.handle == kGpu ? kGpuPool : a.handle == kGpu2 ? kGpuPool2 : kCpuPool}, data);
  return HSA_STATUS_SUCCESS;
}
hsa_status_t f_pool_get_info(hsa_amd_memory_pool_t p, hsa_amd_memory_pool_info_t attr, void* v) {
  if (attr == HSA_AMD_MEMORY_POOL_INFO_LOCATION) {
    *static_cast<hsa_amd_memory_pool_location_t*>(v) =
        p.handle != kCpuPool ? HSA_AMD_MEMORY_POOL_LOCATION_GPU : HSA_AMD_MEMORY_POOL_LOCATION_CPU;
    return HSA_STATUS_SUCCESS;
  }
  if (attr == HSA_AMD_MEMORY_POOL_INFO_SIZE) {
    *static_cast<size_t*>(v) = 288ull << 30;
    return HSA_STATUS_SUCCESS;
  }
  return HSA_STATUS_ERROR_INVALID_ARGUMENT;
}
hsa_status_t f_allocate(hsa_amd_memory_pool_t, size_t, uint32_t, void** ptr) {
  *ptr = reinterpret_cast<void*>(g_next_ptr);
  g_next_ptr += 0x100000;
  return HSA_STATUS_SUCCESS;
}
hsa_status_t f_free(void*) { return HSA_STATUS_SUCCESS; }
hsa_status_t f_vmem_create(hsa_amd_memory_pool_t, size_t, hsa_amd_memory_type_t, uint64_t,
                           hsa_amd_vmem_alloc_handle_t* h) {
  h->handle = g_next_ptr++;
  return HSA_STATUS_SUCCESS;
}
hsa_status_t f_vmem_release(hsa_amd_vmem_alloc_handle_t) { return HSA_STATUS_SUCCESS; }
hsa_queue_t g_queue{};
hsa_status_t f_queue_create(hsa_agent_t, uint32_t, hsa_queue_type32_t, void (*)(hsa_status_t, hsa_queue_t*, void*),
                            void*, uint32_t, uint32_t, hsa_queue_t** q) {
  *q = &g_queue;
  return HSA_STATUS_SUCCESS;
}
int g_destroyed = 0;
hsa_status_t f_queue_destroy(hsa_queue_t*) {
  ++g_destroyed;
  return HSA_STATUS_SUCCESS;
}
hsa_status_t f_cu_set_mask(const hsa_queue_t*, uint32_t bits, const uint32_t* mask) {
  g_last_bits = bits;
  g_last_mask.assign(mask, mask + bits / 32);
  ++g_masks_set;
  return HSA_STATUS_SUCCESS;
}

std::string share_lib() {
  char buf[PATH_MAX];
  ssize_t n = readlink("/proc/self/exe", buf, sizeof buf - 1);
  std::string exe(buf, n > 0 ? static_cast<size_t>(n) : 0);
  return exe.substr(0, exe.rfind('/')) + "/libgpupool_share.so";
}

struct Fake {
  CoreApiTable core{};
  AmdExtTable amd{};
  HsaApiTable table{};
  Fake() {
    core.hsa_iterate_agents_fn = f_iterate_agents;
    core.hsa_agent_get_info_fn = f_agent_get_info;
    core.hsa_queue_create_fn = f_queue_create;
    core.hsa_queue_destroy_fn = f_queue_destroy;
    amd.hsa_amd_agent_iterate_memory_pools_fn = f_iterate_pools;
    amd.hsa_amd_memory_pool_get_info_fn = f_pool_get_info;
    amd.hsa_amd_memory_pool_allocate_fn = f_allocate;
    amd.hsa_amd_memory_pool_free_fn = f_free;
    amd.hsa_amd_vmem_handle_create_fn = f_vmem_create;
    amd.hsa_amd_vmem_handle_release_fn = f_vmem_release;
    amd.hsa_amd_queue_cu_set_mask_fn = f_cu_set_mask;
    table.core_ = &core;
    table.amd_ext_ = &amd;
  }
};

// A private copy of the library: dlopen of the same path would return the instance (and the
// process-wide state) an earlier test already initialised.
void* load_copy(const std::string& dst) {
  std::string cmd = "cp '" + share_lib() + "' '" + dst + "'";
  if (std::system(cmd.c_str()) != 0) return nullptr;
  return dlopen(dst.c_str(), RTLD_NOW | RTLD_LOCAL);
}

// The account file the agent writes (gpupool/agent/agent.py _share_account): 16 KiB, magic,
// limit per GPU; everything else zero.
// Version 2 (``uuids`` given): the account names its GPUs at 8192 + 32 g.
std::string make_account(uint64_t limit, const std::vector<std::string>& uuids = {}) {
  std::string path = "/tmp/gpupool-share-test-" + std::to_string(getpid()) + ".acct";
  std::vector<char> buf(16384, 0);
  std::memcpy(buf.data(), "GPSHARE1", 8);
  std::memcpy(buf.data() + 8, &limit, 8);
  uint32_t ver = uuids.empty() ? 1 : 2, ngpus = uuids.empty() ? 1 : static_cast<uint32_t>(uuids.size());
  std::memcpy(buf.data() + 16, &ver, 4);
  std::memcpy(buf.data() + 20, &ngpus, 4);
  for (size_t g = 0; g < uuids.size(); ++g) std::memcpy(buf.data() + 8192 + 32 * g, uuids[g].c_str(), uuids[g].size());
  int fd = open(path.c_str(), O_CREAT | O_TRUNC | O_RDWR, 0600);
  if (fd < 0 || write(fd, buf.data(), buf.size()) != static_cast<ssize_t>(buf.size())) path.clear();
  if (fd >= 0) close(fd);
  return path;
}

uint64_t account_used(const std::string& path, int gpu = 0) {
  uint64_t v = 0;
  int fd = open(path.c_str(), O_RDONLY);
  if (fd >= 0) {
    if (pread(fd, &v, 8, 64 + 8 * gpu) != 8) v = ~0ull;
    close(fd);
  }
  return v;
}

}  // namespace

TEST(share_lib_budget_and_cu_mask) {
  setenv("GPUPOOL_HBM_LIMIT_BYTES", "1Gi", 1);
  setenv("GPUPOOL_CU_MASK", "0-63,128-159", 1);
  void* lib = dlopen(share_lib().c_str(), RTLD_NOW | RTLD_LOCAL);
  EXPECT_TRUE(lib != nullptr);
  auto on_load = reinterpret_cast<bool (*)(HsaApiTable*, uint64_t, uint64_t, const char* const*)>(dlsym(lib, "OnLoad"));
  auto stats = reinterpret_cast<int (*)(char*, int)>(dlsym(lib, "gpupool_share_stats"));
  EXPECT_TRUE(on_load && stats);

  CoreApiTable core{};
  AmdExtTable amd{};
  core.hsa_iterate_agents_fn = f_iterate_agents;
  core.hsa_agent_get_info_fn = f_agent_get_info;
  core.hsa_queue_create_fn = f_queue_create;
  amd.hsa_amd_agent_iterate_memory_pools_fn = f_iterate_pools;
  amd.hsa_amd_memory_pool_get_info_fn = f_pool_get_info;
  amd.hsa_amd_memory_pool_allocate_fn = f_allocate;
  amd.hsa_amd_memory_pool_free_fn = f_free;
  amd.hsa_amd_vmem_handle_create_fn = f_vmem_create;
  amd.hsa_amd_vmem_handle_release_fn = f_vmem_release;
  amd.hsa_amd_queue_cu_set_mask_fn = f_cu_set_mask;
  HsaApiTable table{};
  table.core_ = &core;
  table.amd_ext_ = &amd;
  EXPECT_TRUE(on_load(&table, 0, 0, nullptr));

  const hsa_amd_memory_pool_t gpu{kGpuPool}, cpu{kCpuPool};
  void *a = nullptr, *b = nullptr, *c = nullptr;
  EXPECT_EQ(amd.hsa_amd_memory_pool_allocate_fn(gpu, 512 * kMi, 0, &a), HSA_STATUS_SUCCESS);
  EXPECT_EQ(amd.hsa_amd_memory_pool_allocate_fn(gpu, 384 * kMi, 0, &b), HSA_STATUS_SUCCESS);
  // 896 MiB live: 256 MiB more would pass 1 GiB
  EXPECT_EQ(amd.hsa_amd_memory_pool_allocate_fn(gpu, 256 * kMi, 0, &c), HSA_STATUS_ERROR_OUT_OF_RESOURCES);
  // system memory is not the slot's HBM
  EXPECT_EQ(amd.hsa_amd_memory_pool_allocate_fn(cpu, 4096 * kMi, 0, &c), HSA_STATUS_SUCCESS);
  uint64_t avail = 0;
  EXPECT_EQ(core.hsa_agent_get_info_fn(hsa_agent_t{kGpu}, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_MEMORY_AVAIL),
                                       &avail),
            HSA_STATUS_SUCCESS);
  EXPECT_EQ(avail, static_cast<uint64_t>(128 * kMi));
  size_t size = 0;
  EXPECT_EQ(amd.hsa_amd_memory_pool_get_info_fn(gpu, HSA_AMD_MEMORY_POOL_INFO_SIZE, &size), HSA_STATUS_SUCCESS);
  EXPECT_EQ(size, static_cast<size_t>(1024 * kMi));
  EXPECT_EQ(amd.hsa_amd_memory_pool_get_info_fn(cpu, HSA_AMD_MEMORY_POOL_INFO_SIZE, &size), HSA_STATUS_SUCCESS);
  EXPECT_EQ(size, static_cast<size_t>(288ull << 30));
  // a free returns its bytes; VMM physical handles count against the same budget
  EXPECT_EQ(amd.hsa_amd_memory_pool_free_fn(a), HSA_STATUS_SUCCESS);
  hsa_amd_vmem_alloc_handle_t h{};
  EXPECT_EQ(amd.hsa_amd_vmem_handle_create_fn(gpu, 512 * kMi, MEMORY_TYPE_NONE, 0, &h), HSA_STATUS_SUCCESS);
  hsa_amd_vmem_alloc_handle_t h2{};
  EXPECT_EQ(amd.hsa_amd_vmem_handle_create_fn(gpu, 256 * kMi, MEMORY_TYPE_NONE, 0, &h2),
            HSA_STATUS_ERROR_OUT_OF_RESOURCES);
  EXPECT_EQ(amd.hsa_amd_vmem_handle_release_fn(h), HSA_STATUS_SUCCESS);
  EXPECT_EQ(amd.hsa_amd_memory_pool_allocate_fn(gpu, 640 * kMi, 0, &c), HSA_STATUS_SUCCESS);

  // every GPU queue gets the slot's CU mask (bits 0-63 and 128-159: 5 words)
  hsa_queue_t* q = nullptr;
  EXPECT_EQ(core.hsa_queue_create_fn(hsa_agent_t{kGpu}, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, 0, 0, &q),
            HSA_STATUS_SUCCESS);
  EXPECT_EQ(g_masks_set, 1);
  EXPECT_EQ(g_last_bits, 160u);
  EXPECT_TRUE(g_last_mask == (std::vector<uint32_t>{~0u, ~0u, 0u, 0u, ~0u}));
  core.hsa_queue_create_fn(hsa_agent_t{kCpu}, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, 0, 0, &q);
  EXPECT_EQ(g_masks_set, 1);  // not on CPU agents
  // an application mask (hipExtStreamCreateWithCUMask) only narrows the slot's
  const uint32_t app[2] = {0x0000FFFFu, 0xFFFFFFFFu};
  amd.hsa_amd_queue_cu_set_mask_fn(&g_queue, 64, app);
  EXPECT_TRUE(g_last_mask == (std::vector<uint32_t>{0x0000FFFFu, ~0u, 0u, 0u, 0u}));
  const uint32_t outside[1] = {0};
  amd.hsa_amd_queue_cu_set_mask_fn(&g_queue, 32, outside);  // nothing left: the slot's mask
  EXPECT_TRUE(g_last_mask == (std::vector<uint32_t>{~0u, ~0u, 0u, 0u, ~0u}));

  char buf[256];
  stats(buf, sizeof buf);
  std::string js(buf);
  EXPECT_TRUE(js.find("\"denied\":2") != std::string::npos);
  EXPECT_TRUE(js.find("\"maskBits\":160") != std::string::npos);
  unsetenv("GPUPOOL_HBM_LIMIT_BYTES");
  unsetenv("GPUPOOL_CU_MASK");
}

// GPUPOOL_SHARE_ACCOUNT: the budget is the pod's, over all its processes. A forked process charges
// the same account; one that dies holding memory (no free ran) has its bytes returned by the next
// process that finds the budget exhausted; a live process's bytes are never taken.
TEST(share_lib_pod_account_across_processes) {
  std::string acct = make_account(1024 * kMi);
  EXPECT_TRUE(!acct.empty());
  setenv("GPUPOOL_HBM_LIMIT_BYTES", "64Gi", 1);  // the account's limit wins
  setenv("GPUPOOL_SHARE_ACCOUNT", acct.c_str(), 1);
  std::string copy = "/tmp/libgpupool_share-test-" + std::to_string(getpid()) + ".so";
  void* lib = load_copy(copy);
  EXPECT_TRUE(lib != nullptr);
  auto on_load = reinterpret_cast<bool (*)(HsaApiTable*, uint64_t, uint64_t, const char* const*)>(dlsym(lib, "OnLoad"));
  auto stats = reinterpret_cast<int (*)(char*, int)>(dlsym(lib, "gpupool_share_stats"));
  Fake f;
  EXPECT_TRUE(on_load(&f.table, 0, 0, nullptr));
  auto alloc = f.amd.hsa_amd_memory_pool_allocate_fn;
  const hsa_amd_memory_pool_t gpu{kGpuPool};
  void *a = nullptr, *b = nullptr;
  EXPECT_EQ(alloc(gpu, 512 * kMi, 0, &a), HSA_STATUS_SUCCESS);
  EXPECT_EQ(account_used(acct), static_cast<uint64_t>(512 * kMi));

  // a second process of the pod: 384 MiB fits, 256 MiB more does not (pod total 1152 > 1024);
  // it then dies without freeing
  pid_t child = fork();
  if (child == 0) {
    void* p = nullptr;
    int rc = alloc(gpu, 384 * kMi, 0, &p) == HSA_STATUS_SUCCESS ? 0 : 1;
    if (alloc(gpu, 256 * kMi, 0, &p) != HSA_STATUS_ERROR_OUT_OF_RESOURCES) rc |= 2;
    _exit(rc);
  }
  int status = 0;
  waitpid(child, &status, 0);
  EXPECT_EQ(WEXITSTATUS(status), 0);
  EXPECT_EQ(account_used(acct), static_cast<uint64_t>(896 * kMi));
  uint64_t avail = 0;
  f.core.hsa_agent_get_info_fn(hsa_agent_t{kGpu}, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_MEMORY_AVAIL),
                               &avail);
  EXPECT_EQ(avail, static_cast<uint64_t>(128 * kMi));  // what the pod has left, not this process

  // over budget -> the dead process's 384 MiB come back first
  EXPECT_EQ(alloc(gpu, 256 * kMi, 0, &b), HSA_STATUS_SUCCESS);
  EXPECT_EQ(account_used(acct), static_cast<uint64_t>(768 * kMi));

  // a live sibling holding 200 MiB is not reclaimed
  int go[2], done[2];
  EXPECT_EQ(pipe(go), 0);
  EXPECT_EQ(pipe(done), 0);
  pid_t live = fork();
  if (live == 0) {
    close(go[0]);
    close(done[1]);  // else the read below never sees EOF
    alarm(20);       // never outlive a broken parent
    void* p = nullptr;
    char c = alloc(gpu, 200 * kMi, 0, &p) == HSA_STATUS_SUCCESS ? 'y' : 'n';
    if (write(go[1], &c, 1) != 1) _exit(3);
    if (read(done[0], &c, 1) < 0) _exit(4);  // hold until the parent says so (EOF)
    _exit(0);
  }
  close(go[1]);
  close(done[0]);
  char c = 0;
  EXPECT_EQ(read(go[0], &c, 1), 1);
  EXPECT_EQ(c, 'y');
  void* d = nullptr;
  EXPECT_EQ(alloc(gpu, 100 * kMi, 0, &d), HSA_STATUS_ERROR_OUT_OF_RESOURCES);
  close(done[1]);
  waitpid(live, &status, 0);
  EXPECT_EQ(alloc(gpu, 100 * kMi, 0, &d), HSA_STATUS_SUCCESS);  // its 200 MiB came back on exit
  EXPECT_EQ(account_used(acct), static_cast<uint64_t>(868 * kMi));

  // frees return bytes to the pod's account
  EXPECT_EQ(f.amd.hsa_amd_memory_pool_free_fn(a), HSA_STATUS_SUCCESS);
  EXPECT_EQ(account_used(acct), static_cast<uint64_t>(356 * kMi));
  char buf[256];
  stats(buf, sizeof buf);
  std::string js(buf);
  EXPECT_TRUE(js.find("\"shared\":1") != std::string::npos);
  EXPECT_TRUE(js.find("\"limit\":1073741824") != std::string::npos);
  EXPECT_TRUE(js.find("\"reclaimed\":" + std::to_string(584 * kMi)) != std::string::npos);
  close(go[0]);
  unlink(acct.c_str());
  unlink(copy.c_str());
  unsetenv("GPUPOOL_HBM_LIMIT_BYTES");
  unsetenv("GPUPOOL_SHARE_ACCOUNT");
}

// Version 2 accounts are keyed by GPU identity, not by each process's enumeration order: a rank that
// sees only GPU B (ROCR_VISIBLE_DEVICES=<B>) and a rank that sees A and B both charge B's counter,
// and a GPU the account does not name is never charged to another GPU's.
TEST(share_lib_account_keyed_by_gpu_uuid) {
  std::string acct = make_account(1024 * kMi, {uuid_of(kGpu), uuid_of(kGpu2)});
  EXPECT_TRUE(!acct.empty());
  setenv("GPUPOOL_HBM_LIMIT_BYTES", "1Gi", 1);
  setenv("GPUPOOL_SHARE_ACCOUNT", acct.c_str(), 1);
  const hsa_amd_memory_pool_t pool_b{kGpuPool2}, pool_a{kGpuPool};
  void* p = nullptr;
  {  // rank 0 sees [A, B]
    g_gpus = {kGpu, kGpu2};
    std::string copy = "/tmp/libgpupool_share-uuid0-" + std::to_string(getpid()) + ".so";
    void* lib = load_copy(copy);
    EXPECT_TRUE(lib != nullptr);
    auto on_load = reinterpret_cast<bool (*)(HsaApiTable*, uint64_t, uint64_t, const char* const*)>(dlsym(lib, "OnLoad"));
    Fake f;
    EXPECT_TRUE(on_load(&f.table, 0, 0, nullptr));
    EXPECT_EQ(f.amd.hsa_amd_memory_pool_allocate_fn(pool_b, 600 * kMi, 0, &p), HSA_STATUS_SUCCESS);
    EXPECT_EQ(f.amd.hsa_amd_memory_pool_allocate_fn(pool_a, 100 * kMi, 0, &p), HSA_STATUS_SUCCESS);
    unlink(copy.c_str());
  }
  EXPECT_EQ(account_used(acct, 0), static_cast<uint64_t>(100 * kMi));
  EXPECT_EQ(account_used(acct, 1), static_cast<uint64_t>(600 * kMi));
  {  // rank 1 sees only B, as its first (ordinal 0) GPU: it must charge B's counter, not A's
    g_gpus = {kGpu2};
    std::string copy = "/tmp/libgpupool_share-uuid1-" + std::to_string(getpid()) + ".so";
    void* lib = load_copy(copy);
    EXPECT_TRUE(lib != nullptr);
    auto on_load = reinterpret_cast<bool (*)(HsaApiTable*, uint64_t, uint64_t, const char* const*)>(dlsym(lib, "OnLoad"));
    Fake f;
    EXPECT_TRUE(on_load(&f.table, 0, 0, nullptr));
    // B holds 600 of its 1024 MiB pod-wide: 500 more is over, 400 fits
    EXPECT_EQ(f.amd.hsa_amd_memory_pool_allocate_fn(pool_b, 500 * kMi, 0, &p), HSA_STATUS_ERROR_OUT_OF_RESOURCES);
    EXPECT_EQ(f.amd.hsa_amd_memory_pool_allocate_fn(pool_b, 400 * kMi, 0, &p), HSA_STATUS_SUCCESS);
    unlink(copy.c_str());
  }
  EXPECT_EQ(account_used(acct, 0), static_cast<uint64_t>(100 * kMi));
  EXPECT_EQ(account_used(acct, 1), static_cast<uint64_t>(1000 * kMi));
  g_gpus = {kGpu};
  unlink(acct.c_str());
  unsetenv("GPUPOOL_HBM_LIMIT_BYTES");
  unsetenv("GPUPOOL_SHARE_ACCOUNT");
}

// The limit the agent fixed lives in a read-only mounted file: a pod that rewrites the limit in
// its (writable) account header, or its env, gains nothing — the smallest limit wins.
TEST(share_lib_read_only_limit_file_wins_over_an_edited_account) {
  std::string acct = make_account(64ull << 30);  // the pod "edited" its account: 64 GiB
  std::string limf = "/tmp/gpupool-share-test-" + std::to_string(getpid()) + ".limit";
  {
    int fd = open(limf.c_str(), O_CREAT | O_TRUNC | O_WRONLY, 0644);
    std::string txt = "GPLIMIT1 " + std::to_string(1024 * kMi) + "\n";
    EXPECT_EQ(write(fd, txt.data(), txt.size()), static_cast<ssize_t>(txt.size()));
    close(fd);
  }
  setenv("GPUPOOL_HBM_LIMIT_BYTES", "128Gi", 1);
  setenv("GPUPOOL_SHARE_ACCOUNT", acct.c_str(), 1);
  setenv("GPUPOOL_SHARE_LIMIT", limf.c_str(), 1);
  std::string copy = "/tmp/libgpupool_share-lim-" + std::to_string(getpid()) + ".so";
  void* lib = load_copy(copy);
  EXPECT_TRUE(lib != nullptr);
  auto on_load = reinterpret_cast<bool (*)(HsaApiTable*, uint64_t, uint64_t, const char* const*)>(dlsym(lib, "OnLoad"));
  Fake f;
  EXPECT_TRUE(on_load(&f.table, 0, 0, nullptr));
  void* p = nullptr;
  const hsa_amd_memory_pool_t gpu{kGpuPool};
  EXPECT_EQ(f.amd.hsa_amd_memory_pool_allocate_fn(gpu, 1000 * kMi, 0, &p), HSA_STATUS_SUCCESS);
  EXPECT_EQ(f.amd.hsa_amd_memory_pool_allocate_fn(gpu, 100 * kMi, 0, &p), HSA_STATUS_ERROR_OUT_OF_RESOURCES);
  unlink(copy.c_str());
  unlink(acct.c_str());
  unlink(limf.c_str());
  unsetenv("GPUPOOL_HBM_LIMIT_BYTES");
  unsetenv("GPUPOOL_SHARE_ACCOUNT");
  unsetenv("GPUPOOL_SHARE_LIMIT");
}

// an application mask that narrows the slot to CUs of ONE XCD (bits 0, 8, 16, 24 with
// 8 XCDs: CU b sits on XCD b % 8) would leave the other XCDs empty, and the driver then silently
// drops the mask — the queue runs on all CUs, the neighbours' included. Such a narrowing falls
// back to the slot's mask; one that keeps a CU on every XCD is applied.
TEST(share_lib_narrowing_that_empties_an_xcd_keeps_the_slot_mask) {
  setenv("GPUPOOL_CU_MASK", "0-127", 1);
  setenv("GPUPOOL_CU_XCDS", "8", 1);
  std::string copy = "/tmp/libgpupool_share-xcd-" + std::to_string(getpid()) + ".so";
  void* lib = load_copy(copy);
  EXPECT_TRUE(lib != nullptr);
  auto on_load = reinterpret_cast<bool (*)(HsaApiTable*, uint64_t, uint64_t, const char* const*)>(dlsym(lib, "OnLoad"));
  auto stats = reinterpret_cast<int (*)(char*, int)>(dlsym(lib, "gpupool_share_stats"));
  Fake f;
  EXPECT_TRUE(on_load(&f.table, 0, 0, nullptr));
  const uint32_t one_xcd[1] = {(1u << 0) | (1u << 8) | (1u << 16) | (1u << 24)};
  f.amd.hsa_amd_queue_cu_set_mask_fn(&g_queue, 32, one_xcd);
  EXPECT_TRUE(g_last_mask == (std::vector<uint32_t>{~0u, ~0u, ~0u, ~0u}));  // the slot's
  const uint32_t every_xcd[1] = {0x000000FFu};  // CUs 0-7: one on each XCD
  f.amd.hsa_amd_queue_cu_set_mask_fn(&g_queue, 32, every_xcd);
  EXPECT_TRUE(g_last_mask == (std::vector<uint32_t>{0xFFu, 0u, 0u, 0u}));
  char buf[320];
  stats(buf, sizeof buf);
  EXPECT_TRUE(std::string(buf).find("\"narrowingsRefused\":1") != std::string::npos);
  unlink(copy.c_str());
  unsetenv("GPUPOOL_CU_MASK");
  unsetenv("GPUPOOL_CU_XCDS");
}

// a pod holding slot 0 on GPU A and slot 1 on GPU B must get slot 0's CUs on A and slot
// 1's on B — not their union on both (which overlaps the sibling tenants). GPUPOOL_CU_MASKS keys
// the masks by the GPU's UUID; a GPU it does not name falls back to GPUPOOL_CU_MASK.
TEST(share_lib_cu_masks_per_gpu_by_uuid) {
  setenv("GPUPOOL_CU_MASKS", "GPU-aaaa000000000001=0-63;GPU-bbbb000000000002=64-127", 1);
  setenv("GPUPOOL_CU_XCDS", "8", 1);
  g_gpus = {kGpu, kGpu2};
  std::string copy = "/tmp/libgpupool_share-pergpu-" + std::to_string(getpid()) + ".so";
  void* lib = load_copy(copy);
  EXPECT_TRUE(lib != nullptr);
  auto on_load = reinterpret_cast<bool (*)(HsaApiTable*, uint64_t, uint64_t, const char* const*)>(dlsym(lib, "OnLoad"));
  Fake f;
  EXPECT_TRUE(on_load(&f.table, 0, 0, nullptr));
  hsa_queue_t* q = nullptr;
  static hsa_queue_t q2;
  EXPECT_EQ(f.core.hsa_queue_create_fn(hsa_agent_t{kGpu}, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, 0, 0, &q),
            HSA_STATUS_SUCCESS);
  EXPECT_TRUE(g_last_mask == (std::vector<uint32_t>{~0u, ~0u}));  // A: 0-63
  // the fake returns the same queue object for every create: give GPU B's queue its own address
  auto make_b = [](hsa_agent_t, uint32_t, hsa_queue_type32_t, void (*)(hsa_status_t, hsa_queue_t*, void*), void*,
                   uint32_t, uint32_t, hsa_queue_t** out) {
    *out = &q2;
    return HSA_STATUS_SUCCESS;
  };
  Fake f2;  // a fresh dispatch table (re-wrapping the wrapped one would recurse)
  f2.core.hsa_queue_create_fn = make_b;
  EXPECT_TRUE(on_load(&f2.table, 0, 0, nullptr));
  EXPECT_EQ(f2.core.hsa_queue_create_fn(hsa_agent_t{kGpu2}, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, 0, 0, &q),
            HSA_STATUS_SUCCESS);
  EXPECT_TRUE(q == &q2);
  EXPECT_TRUE(g_last_mask == (std::vector<uint32_t>{0u, 0u, ~0u, ~0u}));  // B: 64-127
  // an application narrowing on B's queue intersects with B's mask, not A's
  const uint32_t app[4] = {~0u, ~0u, 0x000000FFu, 0u};
  f2.amd.hsa_amd_queue_cu_set_mask_fn(&q2, 128, app);
  EXPECT_TRUE(g_last_mask == (std::vector<uint32_t>{0u, 0u, 0xFFu, 0u}));
  g_gpus = {kGpu};
  unlink(copy.c_str());
  unsetenv("GPUPOOL_CU_MASKS");
  unsetenv("GPUPOOL_CU_XCDS");
}

// queue-map entries are freed on hsa_queue_destroy (a process creating and destroying
// queues for its whole life keeps its per-queue masks), and a queue the map does not know never
// gets the pod-wide union under per-GPU masks (it would overlap sibling tenants).
TEST(share_lib_queue_map_recycles_and_never_widens_unknown_queues) {
  setenv("GPUPOOL_CU_MASKS", "GPU-aaaa000000000001=0-63", 1);
  setenv("GPUPOOL_CU_MASK", "0-127", 1);
  setenv("GPUPOOL_CU_XCDS", "8", 1);
  std::string copy = "/tmp/libgpupool_share-qmap-" + std::to_string(getpid()) + ".so";
  void* lib = load_copy(copy);
  EXPECT_TRUE(lib != nullptr);
  auto on_load = reinterpret_cast<bool (*)(HsaApiTable*, uint64_t, uint64_t, const char* const*)>(dlsym(lib, "OnLoad"));
  static hsa_queue_t pool_q[600];
  static int next_q = 0;
  auto make = [](hsa_agent_t, uint32_t, hsa_queue_type32_t, void (*)(hsa_status_t, hsa_queue_t*, void*), void*,
                 uint32_t, uint32_t, hsa_queue_t** out) {
    *out = &pool_q[next_q++ % 600];
    return HSA_STATUS_SUCCESS;
  };
  Fake f;
  f.core.hsa_queue_create_fn = make;
  EXPECT_TRUE(on_load(&f.table, 0, 0, nullptr));
  const uint32_t app[4] = {0x0000FFFFu, 0u, 0u, 0u};  // narrows to CUs 0-15 (2 per XCD)
  // 600 create/destroy cycles, far past the 256-entry map: every queue still narrows within its
  // own slot's mask (0-63)
  for (int i = 0; i < 600; ++i) {
    hsa_queue_t* q = nullptr;
    EXPECT_EQ(f.core.hsa_queue_create_fn(hsa_agent_t{kGpu}, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, 0, 0, &q),
              HSA_STATUS_SUCCESS);
    g_last_mask.clear();
    f.amd.hsa_amd_queue_cu_set_mask_fn(q, 128, app);
    EXPECT_TRUE(g_last_mask == (std::vector<uint32_t>{0x0000FFFFu, 0u}));
    const int before = g_destroyed;
    f.core.hsa_queue_destroy_fn(q);
    EXPECT_EQ(g_destroyed, before + 1);
  }
  // a queue created outside the library's view: the narrowing is refused, nothing is widened
  static hsa_queue_t stranger;
  const int sets = g_masks_set;
  EXPECT_EQ(f.amd.hsa_amd_queue_cu_set_mask_fn(&stranger, 128, app), HSA_STATUS_SUCCESS);
  EXPECT_EQ(g_masks_set, sets);
  unlink(copy.c_str());
  unsetenv("GPUPOOL_CU_MASKS");
  unsetenv("GPUPOOL_CU_MASK");
  unsetenv("GPUPOOL_CU_XCDS");
}
