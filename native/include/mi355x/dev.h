/* libmi355x_dev — MI355X (gfx950) device discovery, telemetry, health evaluation and
 * topology-aware selection, behind a C ABI (loaded by the node agent via ctypes).
 *
 * Replaces the reference's Azure SDK calls (README.md:179-221) as the thing the provider layer
 * talks to: instead of listing/creating/deleting VMs it enumerates physical GPUs and reports the
 * facts readiness is derived from (xGMI link state, HBM ECC, thermals, partition mode).
 *
 * Backends:
 *   "amdsmi"  libamd_smi.so (dlopen'ed; ROCm 7.x) — the production path;
 *   "cli"     `amd-smi ... --json` subprocess parsing — an independent path for cross-checks;
 *   "fake"    a JSON fixture (tests/fixtures/node_8x_mi355x.json), for CPU-only testing;
 *   "auto"    amdsmi if it initialises and finds a GPU, else error.
 * Any backend accepts a fault-overlay file (hot-reloaded on mtime change) that is deep-merged
 * into every snapshot — SURVEY.md §5 "Fault injection".
 *
 * All strings returned are heap-allocated JSON; release with mi355x_free().
 */
#ifndef MI355X_DEV_H_
#define MI355X_DEV_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mi355x_dev mi355x_dev;

/* config_json: {"fixture": path, "faults": path, "amdsmi_bin": "amd-smi", "node": name}.
 * Returns NULL on failure with a message in err. */
mi355x_dev* mi355x_dev_open(const char* backend, const char* config_json, char* err, size_t errlen);
void mi355x_dev_close(mi355x_dev* d);

/* Node snapshot: {"backend","node","ts","devices":[...],"topology":{"weights":[[..]],"types":[[..]]}} */
char* mi355x_dev_snapshot(mi355x_dev* d);

/* Health-only snapshot: per device {index, uuid, ecc, xgmi, temps, present} (+ fault overlay),
 * cheap enough for a ~10 Hz poll; same shape as the corresponding fields of the full snapshot. */
char* mi355x_dev_health_snapshot(mi355x_dev* d);

/* Health verdict for one device snapshot against a pool policy and the ECC baseline taken at
 * claim time: {"healthy","present","xgmiOk","eccOk","thermalOk","partitionOk","reasons":[...]} */
char* mi355x_dev_evaluate(const char* device_json, const char* baseline_json, const char* policy_json);

/* Many verdicts in one call: items [{"device", "baseline" (default: the device), "policy"}] ->
 * [verdict, ...] in order (the agent evaluates every GPU on each health poll). */
char* mi355x_dev_evaluate_batch(const char* items_json);

/* Topology-aware all-or-nothing selection.
 * req: {"count":k,"candidates":[idx..],"owned":[idx..],"policy":"xgmi-packed"|"any",
 *       "weights":[[..]],"numa":[..]} -> {"selected":[idx..]} ("selected" empty if < k). */
char* mi355x_dev_select(const char* request_json);

/* Hardware event source (amdsmi event notification: ThermalThrottle, GPUPreReset, GPUPostReset,
 * VMFault). Blocks up to timeout_ms: {"supported": bool, "events": [{"index","type","message"}]}.
 * supported=false returns at once (fake/cli backends, or the driver refused the subscription). */
char* mi355x_dev_wait_events(mi355x_dev* d, int timeout_ms);

/* Fault-overlay watch (inotify): blocks up to timeout_ms for the overlay file to be rewritten,
 * moved into place or deleted: {"supported": bool, "changed": bool}. */
char* mi355x_dev_wait_faults(mi355x_dev* d, int timeout_ms);

void mi355x_free(char* p);
const char* mi355x_dev_version(void);

#ifdef __cplusplus
}
#endif

#endif /* MI355X_DEV_H_ */
