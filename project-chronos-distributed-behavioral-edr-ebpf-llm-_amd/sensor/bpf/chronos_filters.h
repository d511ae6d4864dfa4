/* chronos_filters.h — the sensor's in-kernel noise policy, shared by the eBPF program and the host build.
 *
 * Behavioural contract (reference chronos_sensor.py:28-47 helpers, :74-92 policy):
 *   an OPEN event is dropped in the kernel when its path
 *     - starts with one of  /lib /usr/lib /usr/share /etc/ssl /etc/fonts /etc/host /dev/ /proc/
 *     - or ends with one of .so .cache .mo .conf .crt .curlrc
 *   EXEC events are never filtered (chronos_sensor.py:50-64).
 *
 * Unlike the reference, which re-counts strlen(path) inside every suffix test (6 x 256 iterations per openat),
 * the length is computed once and the policy is expressed as X-macro tables, so the same lists drive
 *   (a) the BPF program  (sensor/bpf/chronos.bpf.c, compiled by BCC/clang at load time),
 *   (b) the C++ host library (csrc/sensor_host/sensor_host.cpp) used for replay, benchmarking and tests.
 * All loops are bounded by compile-time constants so the BPF verifier accepts them.
 *
 * CHRONOS_FILTER_STRICT (opt-in) adds /etc/localtime and any *curlrc path.
 */
#ifndef CHRONOS_FILTERS_H
#define CHRONOS_FILTERS_H

#define CHRONOS_COMM_LEN 16   /* TASK_COMM_LEN */
#define CHRONOS_PATH_LEN 256  /* data_t.argv */
#define CHRONOS_TYPE_LEN 10   /* data_t.type */
#define CHRONOS_PREFIX_SCAN 20 /* max prefix chars compared (reference starts_with bound) */
#define CHRONOS_SUFFIX_SCAN 10 /* max suffix chars (reference ends_with bound) */

#ifdef __cplusplus
#define CHRONOS_FN static inline
#else
#define CHRONOS_FN static inline __attribute__((always_inline))
#endif

/* Policy tables.  X(literal) is expanded once per entry. */
#define CHRONOS_NOISE_PREFIXES(X) \
    X("/lib") X("/usr/lib") X("/usr/share") X("/etc/ssl") X("/etc/fonts") X("/etc/host") X("/dev/") X("/proc/")
#define CHRONOS_NOISE_SUFFIXES(X) \
    X(".so") X(".cache") X(".mo") X(".conf") X(".crt") X(".curlrc")
#define CHRONOS_STRICT_PREFIXES(X) X("/etc/localtime")
#define CHRONOS_STRICT_SUFFIXES(X) X("curlrc")

/* Bounded strlen over a NUL-terminated buffer of at most CHRONOS_PATH_LEN bytes. */
CHRONOS_FN int chronos_path_len(const char *s) {
    int n = 0;
#pragma unroll
    for (int i = 0; i < CHRONOS_PATH_LEN; i++) {
        if (s[i] == 0) break;
        n++;
    }
    return n;
}

/* 1 if s begins with prefix p (compares at most CHRONOS_PREFIX_SCAN chars, like the reference). */
CHRONOS_FN int chronos_has_prefix(const char *s, const char *p) {
#pragma unroll
    for (int i = 0; i < CHRONOS_PREFIX_SCAN; i++) {
        if (p[i] == 0) return 1;
        if (s[i] != p[i]) return 0;
    }
    return 1;
}

/* 1 if the first slen bytes of s end with suffix p (suffix at most CHRONOS_SUFFIX_SCAN chars). */
CHRONOS_FN int chronos_has_suffix(const char *s, int slen, const char *p) {
    int plen = 0;
#pragma unroll
    for (int i = 0; i < CHRONOS_SUFFIX_SCAN; i++) {
        if (p[i] == 0) break;
        plen++;
    }
    if (plen > slen) return 0;
    int base = slen - plen;
#pragma unroll
    for (int i = 0; i < CHRONOS_SUFFIX_SCAN; i++) {
        if (i >= plen) break;
        int j = base + i;
        if (j < 0 || j >= CHRONOS_PATH_LEN) return 0; /* verifier: keep the index provably in range */
        if (s[j] != p[i]) return 0;
    }
    return 1;
}

#define CHRONOS_X_PREFIX(lit) if (chronos_has_prefix(path, lit)) return 1;
#define CHRONOS_X_SUFFIX(lit) if (chronos_has_suffix(path, n, lit)) return 1;

/* 1 if an OPEN of `path` is filesystem noise that the kernel program drops before perf_submit. */
CHRONOS_FN int chronos_open_is_noise(const char *path) {
    CHRONOS_NOISE_PREFIXES(CHRONOS_X_PREFIX)
    int n = chronos_path_len(path);
    CHRONOS_NOISE_SUFFIXES(CHRONOS_X_SUFFIX)
#ifdef CHRONOS_FILTER_STRICT
    CHRONOS_STRICT_PREFIXES(CHRONOS_X_PREFIX)
    CHRONOS_STRICT_SUFFIXES(CHRONOS_X_SUFFIX)
#endif
    return 0;
}

/* Host-side runtime switch for the strict list (the BPF build selects it with -DCHRONOS_FILTER_STRICT). */
CHRONOS_FN int chronos_open_is_noise_strict(const char *path) {
    if (chronos_open_is_noise(path)) return 1;
    CHRONOS_STRICT_PREFIXES(CHRONOS_X_PREFIX)
    int n = chronos_path_len(path);
    CHRONOS_STRICT_SUFFIXES(CHRONOS_X_SUFFIX)
    return 0;
}

#undef CHRONOS_X_PREFIX
#undef CHRONOS_X_SUFFIX

#endif /* CHRONOS_FILTERS_H */
