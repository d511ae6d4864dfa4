/* chronos.bpf.c — CHRONOS kernel sensor (BCC dialect).
 *
 * Loaded by sensor/loader.py with  BPF(src_file=<this>, cflags=["-I<bpf dir>"]).
 * Hooks (reference chronos_sensor.py:50-103):
 *   kprobe on the arch execve symbol -> syscall__execve : one EXEC record, argv[0] of the new image,
 *                                                         comm = the *pre-exec* image name, never filtered
 *   kprobe on the arch openat symbol -> syscall__openat : one OPEN record unless chronos_open_is_noise(path)
 * Records are the 288-byte struct data_t below (ABI mirrored by sensor/abi.py and csrc/sensor_host), pushed to the
 * per-CPU perf array `events` (the reference's transport, chronos_sensor.py:25,95) or, built with
 * -DCHRONOS_RINGBUF=<pages>, to ONE BPF ring buffer shared by all CPUs (kernel >= 5.8): records then reach user space
 * in global submission order instead of drained CPU by CPU (the out-of-order PIDs of the reference screenshot,
 * SURVEY.md §3.4), with no per-CPU over-provisioning and exact-size samples (no PERF_SAMPLE_RAW padding).
 */
#include <uapi/linux/ptrace.h>
#include <linux/sched.h>
#include <linux/fs.h>

#include "chronos_filters.h"

struct data_t {
    u32 pid;                      /* TGID (bpf_get_current_pid_tgid() >> 32) */
    char comm[TASK_COMM_LEN];     /* 16 */
    char argv[CHRONOS_PATH_LEN];  /* 256: argv[0] for EXEC, path for OPEN */
    char type[CHRONOS_TYPE_LEN];  /* "EXEC" / "OPEN", NUL padded; 2 bytes of tail padding follow */
};

#ifdef CHRONOS_RINGBUF
BPF_RINGBUF_OUTPUT(events, CHRONOS_RINGBUF);
#define CHRONOS_SUBMIT(ctx, d) events.ringbuf_output((d), sizeof(*(d)), 0)
#else
BPF_PERF_OUTPUT(events);
#define CHRONOS_SUBMIT(ctx, d) events.perf_submit((ctx), (d), sizeof(*(d)))
#endif

static inline __attribute__((always_inline)) void chronos_fill_task(struct data_t *d) {
    d->pid = bpf_get_current_pid_tgid() >> 32;
    bpf_get_current_comm(&d->comm, sizeof(d->comm));
}

int syscall__execve(struct pt_regs *ctx, const char __user *filename,
                    const char __user *const __user *argv) {
    struct data_t d = {};
    chronos_fill_task(&d);
    const char *arg0 = NULL;
    bpf_probe_read_user(&arg0, sizeof(arg0), &argv[0]);
    if (arg0)
        bpf_probe_read_user_str(&d.argv, sizeof(d.argv), arg0);
    __builtin_memcpy(&d.type, "EXEC", 5);
    CHRONOS_SUBMIT(ctx, &d);
    return 0;
}

int syscall__openat(struct pt_regs *ctx, int dfd, const char __user *filename, int flags) {
    struct data_t d = {};
    bpf_probe_read_user_str(&d.argv, sizeof(d.argv), filename);
    if (chronos_open_is_noise(d.argv))
        return 0;                 /* dropped in kernel: no user-space wake-up */
    chronos_fill_task(&d);
    __builtin_memcpy(&d.type, "OPEN", 5);
    CHRONOS_SUBMIT(ctx, &d);
    return 0;
}
