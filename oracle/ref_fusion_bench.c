/*
 * oracle/ref_fusion_bench.c -- one pinned CPU-baseline worker: the REFERENCE engine lib/fusion.c timed with the
 * t/ptlsbench.c methodology.
 *
 * BASELINE INFRASTRUCTURE ONLY.  oracle/Makefile links this file with the unmodified /root/reference/lib/fusion.c
 * and lib/picotls.c (flags of CMakeLists.txt:158) into oracle/_ref/ref_fusion_bench.  bench.py's cpu_baseline leg starts one process
 * per core (before it touches the GPU), each pinned to its core, and sums them.  Nothing in rapido_amd/ uses it.
 *
 * Methodology of bench_run_one (t/ptlsbench.c:80-165): batches of 1000 records; all encryptions of a batch, then
 * all decryptions; the AAD is the 32-byte h[4] whose h[0] is the record sequence number, which is also the
 * nonce's seq (t/ptlsbench.c:87,117-122,127-133); the output buffers are touched before timing (ptlsbench's
 * first batch pays the page faults of v_enc, t/ptlsbench.c:101-106); time is CLOCK_PROCESS_CPUTIME_ID
 * (t/ptlsbench.c:59-73); Mbps = 8 L N / us (t/ptlsbench.c:167-175).  The engine is driven through its direct API
 * with capacity L + 32 (ptls_fusion_aesgcm_new, lib/fusion.c:775), because through the AEAD slot every record
 * above ~1500 B gets an undefined tag (set_capacity, lib/fusion.c:808) and ptlsbench's
 * decrypt check then fails.  The nonce is built as the slot does (calc_counter, lib/fusion.c:898-905).
 *
 *   ref_fusion_bench KEYLEN LEN NRECORDS CPU   (CPU < 0: not pinned)
 * prints one JSON line: CPU-time and wall-clock rates of this process.
 */
#ifndef _GNU_SOURCE
#define _GNU_SOURCE
#endif
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <immintrin.h>
#include "picotls.h"
#include "picotls/fusion.h"

#define BATCH 1000

static uint64_t clock_us(clockid_t c)
{
    struct timespec ts;
    clock_gettime(c, &ts);
    return (uint64_t)ts.tv_sec * 1000000u + (uint64_t)ts.tv_nsec / 1000u;
}

/* calc_counter (lib/fusion.c:898-905): static IV xor BE64(seq), byte-swapped into an __m128i */
static __m128i counter_for(const uint8_t iv[12], uint64_t seq)
{
    uint8_t n[16] = {0};
    memcpy(n, iv, 12);
    for (int i = 0; i < 8; ++i)
        n[4 + i] ^= (uint8_t)(seq >> (56 - 8 * i));
    const __m128i bswap = _mm_set_epi8(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    return _mm_shuffle_epi8(_mm_loadu_si128((const __m128i *)n), bswap);
}

int main(int argc, char **argv)
{
    if (argc != 5) {
        fprintf(stderr, "usage: %s KEYLEN LEN NRECORDS CPU\n", argv[0]);
        return 2;
    }
    const size_t keylen = (size_t)atoi(argv[1]), l = (size_t)atol(argv[2]), n = (size_t)atol(argv[3]);
    const int cpu = atoi(argv[4]);
    if ((keylen != 16 && keylen != 32) || n == 0)
        return 2;
    if (cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(cpu, &set);
        if (sched_setaffinity(0, sizeof(set), &set) != 0) {
            perror("sched_setaffinity");
            return 3;
        }
    }
    if (!ptls_fusion_is_supported_by_cpu()) {
        printf("{\"error\": \"cpu lacks AES-NI/PCLMUL/AVX2\"}\n");
        return 4;
    }
    uint8_t key[32], iv[12];
    memset(key, 'z', sizeof(key));
    memset(iv, 'y', sizeof(iv));
    ptls_fusion_aesgcm_context_t *ctx = ptls_fusion_aesgcm_new(key, keylen, l + 32);
    uint8_t *v_in = calloc(1, l + 1), *v_dec = calloc(1, l + 16);
    uint8_t *v_enc[BATCH];
    for (int i = 0; i < BATCH; ++i) {
        v_enc[i] = malloc(l + 16);
        memset(v_enc[i], 0, l + 16);
    }
    uint64_t h[4] = {0, 0, 0, 0}, s = 0, t_enc = 0, t_dec = 0;
    int failed = 0;
    const uint64_t w0 = clock_us(CLOCK_MONOTONIC);
    for (size_t k = 0; k < n && !failed;) {
        const size_t imax = n - k > BATCH ? BATCH : n - k;
        const uint64_t old_h = h[0], t0 = clock_us(CLOCK_PROCESS_CPUTIME_ID);
        for (size_t i = 0; i < imax; ++i) {
            h[0]++;
            ptls_fusion_aesgcm_encrypt(ctx, v_enc[i], v_in, l, counter_for(iv, h[0]), h, sizeof(h), NULL);
            s += v_enc[i][l];
        }
        const uint64_t t1 = clock_us(CLOCK_PROCESS_CPUTIME_ID);
        h[0] = old_h;
        for (size_t i = 0; i < imax; ++i) {
            h[0]++;
            if (!ptls_fusion_aesgcm_decrypt(ctx, v_dec, v_enc[i], l, counter_for(iv, h[0]), h, sizeof(h), v_enc[i] + l)) {
                failed = 1;
                break;
            }
            s += v_dec[0];
        }
        const uint64_t t2 = clock_us(CLOCK_PROCESS_CPUTIME_ID);
        t_enc += t1 - t0;
        t_dec += t2 - t1;
        k += imax;
    }
    const uint64_t wall = clock_us(CLOCK_MONOTONIC) - w0;
    const double bytes = (double)l * (double)n, gib = 1024.0 * 1024.0 * 1024.0;
    printf("{\"cpu\": %d, \"keylen\": %zu, \"len\": %zu, \"n\": %zu, \"encrypt_us\": %llu, \"decrypt_us\": %llu, "
           "\"wall_us\": %llu, \"encrypt_mbps\": %.1f, \"decrypt_mbps\": %.1f, \"seal_gibps\": %.4f, \"open_gibps\": %.4f, "
           "\"failed\": %d, \"checksum\": %llu}\n",
           cpu, keylen, l, n, (unsigned long long)t_enc, (unsigned long long)t_dec, (unsigned long long)wall,
           8.0 * bytes / (double)(t_enc ? t_enc : 1), 8.0 * bytes / (double)(t_dec ? t_dec : 1),
           bytes / ((double)(t_enc ? t_enc : 1) * 1e-6) / gib, bytes / ((double)(t_dec ? t_dec : 1) * 1e-6) / gib, failed,
           (unsigned long long)s);
    for (int i = 0; i < BATCH; ++i)
        free(v_enc[i]);
    free(v_in);
    free(v_dec);
    ptls_fusion_aesgcm_free(ctx);
    return failed ? 1 : 0;
}
