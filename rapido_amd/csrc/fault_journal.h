/*
 * fault_journal.h -- the engine's record of its recent device work, reported when the GPU signals a memory fault
 * (fault_journal.c).  Internal to the library: the public entry points are in include/ptls_mi355x.h ("diagnostics").
 */
#ifndef PTLS_MI355X_FAULT_JOURNAL_H
#define PTLS_MI355X_FAULT_JOURNAL_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

/* a pointer argument of a launch: [p, p + len), len 0 when the extent is the caller's (an arena base) */
typedef struct {
    const char *name;
    const void *p;
    uint64_t len;
} ptls_mi355x_journal_arg_t;

#define PTLS_MI355X_JOURNAL_ARGS 8

/* one kernel launch on `stream` (grid blocks x threads over n records) with its pointer arguments */
void ptls_mi355x_journal_launch(const char *kernel, const void *stream, uint32_t blocks, uint32_t threads, uint64_t n,
                                const ptls_mi355x_journal_arg_t *args, size_t nargs);

/* a device memory event (allocation, free, host registration, device check) over [p, p + len) */
void ptls_mi355x_fault_journal_note(const char *what, const void *p, size_t len);

/* a table printed in every fault report (e.g. the record layer's host registrations); it must not block: called from
 * the runtime's event thread while other threads may hold the library's locks */
typedef void (*ptls_mi355x_journal_dumper_t)(FILE *f, uint64_t va);
void ptls_mi355x_fault_journal_add_dumper(ptls_mi355x_journal_dumper_t fn);

#ifdef __cplusplus
}
#endif

#endif
