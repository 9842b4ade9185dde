/*
 * psg_records.h — on-disk result records of the batched HO executor (".psgr").
 *
 * the executor as a bug-finder needs results that outlive
 * the process — sampled per-instance results of a run, and counterexamples
 * found by the adversary search (round_amd/adversary.py) together with the
 * exact schedule and inputs that replay them (psg_load_schedule +
 * psg_load_inputs + psg_run_batch, or the CPU oracle, or an in-JVM harness).
 *
 * The reference has no counterpart: its results are the `ConsensusIO.decide`
 * callbacks (e.g. example/Otr.scala:68-70) and log lines
 * (psync/runtime/InstanceHandler.scala:248-257); the Spec is only checked
 * symbolically (psync/verification/Verifier.scala:111-275).
 *
 * Layout (all little-endian, all offsets from the start of the file):
 *
 *   psg_rec_header                     (fixed size, PSG_REC_HEADER_BYTES)
 *   section payloads                   (each aligned to PSG_REC_ALIGN bytes)
 *
 * Every array section is row-major over the instances listed in the IDS
 * section (count rows). Readers locate sections by kind; unknown kinds are
 * skipped, so later versions may add sections without breaking readers.
 * A Python reader/writer is round_amd/records.py; this header is what a C or
 * JNI reader needs (no library call is required to read a file).
 */
#ifndef PSG_RECORDS_H
#define PSG_RECORDS_H

#include <stdint.h>
#include <string.h>

#include "psg.h"

#ifdef __cplusplus
extern "C" {
#endif

#define PSG_REC_MAGIC "PSGREC\r\n" /* 8 bytes, no terminator in the file */
#define PSG_REC_VERSION 2u /* 2: psg_config of ABI 4 (device list) */
#define PSG_REC_ALIGN 64u
#define PSG_REC_MAX_SECTIONS 16
#define PSG_REC_NAME_BYTES 24

enum psg_rec_kind {
  PSG_REC_IDS = 1,          /* uint64 [count]                global instance ids */
  PSG_REC_SUMMARY = 2,      /* psg_instance_summary [count]  (24 B each, psg.h) */
  PSG_REC_INIT_I32 = 3,     /* int32 [count][n]              initial values (ConsensusIO.initialValue) */
  PSG_REC_INIT_F64 = 4,     /* double [count][n]             initial values (RealConsensusIO) */
  PSG_REC_HO = 5,           /* uint64 [count][R][n][W]       explicit HO sets (psg_load_schedule layout) */
  PSG_REC_CRASH = 6,        /* int32 [count][n]              crash rounds, -1 = correct */
  PSG_REC_PROCESS = 7,      /* psg_process_record [count][n] (16 B each, psg.h) */
  PSG_REC_DECISION_F64 = 8, /* double [count][n]             Double decisions (EpsilonConsensus) */
  PSG_REC_META = 9          /* UTF-8 JSON object             provenance (search target, predicate, ...) */
};

typedef struct psg_rec_section {
  uint32_t kind;       /* enum psg_rec_kind */
  uint32_t elem_bytes; /* bytes per element (1 for META) */
  uint64_t offset;     /* file offset of the payload (multiple of PSG_REC_ALIGN) */
  uint64_t nbytes;     /* payload bytes */
} psg_rec_section;     /* 24 bytes */

typedef struct psg_rec_header {
  char magic[8];          /* PSG_REC_MAGIC */
  uint32_t version;       /* PSG_REC_VERSION */
  uint32_t header_bytes;  /* sizeof(psg_rec_header) */
  psg_config cfg;         /* the configuration the records were produced under (psg.h) */
  uint64_t count;         /* instances (rows) */
  uint32_t n_sections;    /* used entries of sections[] */
  uint32_t n_slots;       /* check slots (psg_check_count, or a Spec program's slot count) */
  char slot_names[PSG_MAX_CHECKS][PSG_REC_NAME_BYTES]; /* NUL-padded, slot order of first_fail */
  char class_name[64];    /* reference class name, e.g. "example.OTR" (NUL-padded) */
  psg_rec_section sections[PSG_REC_MAX_SECTIONS];
} psg_rec_header;

#define PSG_REC_HEADER_BYTES ((uint32_t)sizeof(psg_rec_header))

/* 0 if h looks like a header of this version, else PSG_EINVAL. */
static inline int psg_rec_check_header(const psg_rec_header* h) {
  if (memcmp(h->magic, PSG_REC_MAGIC, 8) != 0) return PSG_EINVAL;
  if (h->version != PSG_REC_VERSION || h->header_bytes != PSG_REC_HEADER_BYTES) return PSG_EINVAL;
  if (h->n_sections > PSG_REC_MAX_SECTIONS || h->n_slots > PSG_MAX_CHECKS) return PSG_EINVAL;
  return 0;
}

/* The section of a kind, or NULL. */
static inline const psg_rec_section* psg_rec_find(const psg_rec_header* h, uint32_t kind) {
  for (uint32_t i = 0; i < h->n_sections && i < PSG_REC_MAX_SECTIONS; ++i)
    if (h->sections[i].kind == kind) return &h->sections[i];
  return (const psg_rec_section*)0;
}

#ifdef __cplusplus
}
#endif

#endif /* PSG_RECORDS_H */
