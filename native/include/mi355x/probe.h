/* libmi355x_probe — HIP readiness probe for MI355X (gfx950). See native/src/probe/probe.hip.
 *
 * The node agent loads this once (ctypes) and calls mi355x_probe_init() at start-up so every
 * device context is warm; a claim-time probe then costs only its kernels (HBM pattern
 * fill/verify + bf16 MFMA GEMM checks), not HIP runtime initialisation.
 * Device indices are HIP ordinals within the calling process's visible set.
 */
#ifndef MI355X_PROBE_H_
#define MI355X_PROBE_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Returns the number of HIP devices (>= 0) or -1 with a message in err. Idempotent. */
int mi355x_probe_init(char* err, size_t errlen);
int mi355x_probe_device_count(void);
/* {"device","hipUUID","name","gcnArch","bdf","totalMem","computeUnits"} */
char* mi355x_probe_identify(int device);
/* opts: {"hbmBytes":1073741824,"patterns":2,"mfma":true,"gemmN":4096,"gemmReps":3,
 *        "requireAllCUs":true}
 * -> {"passed":bool,"hbm":{...,"GBps"},"mfma":{...,"tflops"},
 *     "cus":{"expected","mfmaVerified","perXcd":[8],"gemmTiles","badWaves","ok"},"ms":...}
 * cus: every CU's matrix cores are exercised by a census kernel (chained MFMAs checked exactly per
 * wave, the CU identified by its XCC_ID/HW_ID registers); with requireAllCUs the probe fails
 * unless mfmaVerified >= the runtime's CU count. gemmTiles = CUs that ran tiles of the timed GEMM. */
char* mi355x_probe_run(int device, const char* opts_json);
/* xGMI peer check: src writes a pattern, copies it to dst over the peer link
 * (hipMemcpyPeerAsync after hipDeviceEnablePeerAccess), dst verifies every bit.
 * opts: {"bytes":268435456}. src == dst runs the same path as a local device copy.
 * -> {"src","dst","canAccessPeer":bool,"passed":bool,"badBits","GBps","ms"} */
char* mi355x_probe_peer(int src, int dst, const char* opts_json);
/* The whole ring at once: link i copies devs[i] -> devs[(i+1) % n], all links concurrently (each
 * GPU pair of an MI355X node has its own xGMI link), then every receiver verifies. Send / receive
 * windows are kept between calls and freed with the idle arena. A device may repeat ([0, 0] on a
 * 1-GPU box runs local copies through the same path). opts: {"bytes":67108864}
 * -> {"bytes","links":[{"src","dst","canAccessPeer","passed","badBits","bytes","GBps","ms"}],
 *     "passed":bool} */
char* mi355x_probe_peer_ring(const int* devs, int n, const char* opts_json);
/* One window of the rotating HBM sweep: a buffer of all free HBM minus "reserve" bytes is
 * allocated (kept across calls while "keep" is true; released by mi355x_probe_sweep_release) and
 * [offset, offset+bytes) of it is pattern-tested in both polarities.
 * opts: {"offset":0,"bytes":17179869184,"reserve":4294967296,"keep":false,"injectBitFlips":0}
 * -> {"passed","offset","bytes","span","badBits","firstBadOffset","GBps","ms","allocMs"} */
char* mi355x_probe_hbm_sweep(int device, const char* opts_json);
/* Allocate / free the sweep buffer without holding the device's probe lock (allocating ~282 GiB
 * takes ~0.4 s and freeing it ~2.9 s on MI355X: a claim-time probe must never wait for either).
 * alloc: 1 = allocated, 0 = already held, <0 = error. Both work in 1 GiB chunks and wait between
 * chunks while a claim-time probe of the device runs. release: 1 = freed, 0 = none held. */
int mi355x_probe_sweep_alloc(int device, long long reserve_bytes);
int mi355x_probe_sweep_release(int device);
/* The probe's production GEMM (256x256x64 MFMA tile) on caller HOST buffers (copied in and out):
 * C[m][n] (fp32) = A[m][k] (bf16, row-major) * Bt[n][k]^T (bf16, row-major). m, n multiples of
 * 256, k of 64. For independent numerics checks against a CPU torch.matmul (torch bundles its own
 * HIP runtime, so device pointers cannot be shared with it in one process). 0 = ok. */
int mi355x_probe_gemm_bf16(int device, const void* A, const void* Bt, void* C, int m, int n, int k);
void mi355x_probe_free(char* p);

#ifdef __cplusplus
}
#endif

#endif /* MI355X_PROBE_H_ */
