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
/* opts: {"hbmBytes":1073741824,"patterns":2,"mfma":true,"gemmN":4096,"gemmReps":3}
 * -> {"passed":bool,"hbm":{...,"GBps"},"mfma":{...,"tflops"},"ms":...} */
char* mi355x_probe_run(int device, const char* opts_json);
/* xGMI peer check: src writes a pattern, copies it to dst over the peer link
 * (hipMemcpyPeerAsync after hipDeviceEnablePeerAccess), dst verifies every bit.
 * opts: {"bytes":268435456}. src == dst runs the same path as a local device copy.
 * -> {"src","dst","canAccessPeer":bool,"passed":bool,"badBits","GBps","ms"} */
char* mi355x_probe_peer(int src, int dst, const char* opts_json);
void mi355x_probe_free(char* p);

#ifdef __cplusplus
}
#endif

#endif /* MI355X_PROBE_H_ */
