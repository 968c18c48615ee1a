/*
 * pcabi_oracle.h -- CPU ORACLE for the Porechop_ABI adapter-alignment hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This is a plain-C restatement of the reference algorithm
 * (reference: porechop_abi/src/adapter_align.cpp + alignment.cpp + vendored SeqAn 2.4.0
 * globalAlignment / AlignConfig<1,1,1,1>). It is used by tests/, __graft_entry__.smoke()
 * and the cpu_baseline leg of bench.py as the CHECKER. The product library
 * (custom_porechop_abi_amd/libpcabi.so) never links or calls it.
 *
 * Parity pinning: tests/golden/ holds result strings produced by the reference itself
 * (oracle/_ref/cpp_functions.so compiled from /root/reference sources by oracle/Makefile),
 * and tests/test_oracle_golden.py checks this restatement against every vector.
 */
#ifndef PCABI_ORACLE_H
#define PCABI_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* Same fields ScoredAlignment computes (porechop_abi/include/alignment.h:19-27), plus the
 * integer numerators / denominators of the two identities so callers can reproduce the
 * "%f" text exactly. rs == -1 means "no alignment" (empty read or adapter). */
typedef struct {
    int rs, re, as, ae;     /* read start / end (inclusive), adapter start / end      */
    int score;              /* raw DP score (SeqAn globalAlignment return value)      */
    int m;                  /* matching columns (identical for both identities)       */
    int l1;                 /* aligned-region length; 0 -> pid1 is NaN ("-nan")        */
    int l2;                 /* full-adapter span length                               */
} pcabi_oracle_result;

/* Align one read (horizontal sequence) against one adapter (vertical sequence).
 * Scoring arguments in Python order: (match, mismatch, gap_open, gap_extend). */
void pcabi_oracle_align(const char *read, int n, const char *adapter, int l,
                        int match, int mismatch, int gap_open, int gap_extend,
                        pcabi_oracle_result *out);

/* Byte-compatible restatement of adapterAlignment(): malloc'd "rs,re,as,ae,score,pid1,pid2". */
char *pcabi_oracle_adapter_alignment(const char *read, const char *adapter,
                                     int match, int mismatch, int gap_open, int gap_extend);
void pcabi_oracle_free(char *p);

/* Batch helper for the CPU baseline: n_pairs alignments, windows packed back to back.
 * read_off[p], read_len[p] index into reads; adp_idx[p] selects adapter (adp_off/adp_len).
 * Results written as 8 int32 per pair: rs,re,as,ae,score,m,l1,l2. */
void pcabi_oracle_align_batch(const char *reads, const long long *read_off, const int *read_len,
                              const char *adapters, const int *adp_off, const int *adp_len,
                              const int *adp_idx, long long n_pairs,
                              int match, int mismatch, int gap_open, int gap_extend,
                              int *results);

/* check_compatibility restated (ab-initio clustering link test): 0 / 1 / 2, or -1 where the
 * reference has no defined result (an empty sequence, or no overlap: division by zero). */
int pcabi_oracle_compat(const char *s1, const char *s2);

#ifdef __cplusplus
}
#endif
#endif
