/*
 * tci_oracle.h -- shared declarations of the CPU oracle (TEST INFRASTRUCTURE ONLY: loaded by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline legs; never by the product).
 */
#ifndef TCI_ORACLE_H_
#define TCI_ORACLE_H_

#include <stdint.h>

typedef struct {
  double L0;
  int32_t n_seg;
  const double *ms2_start, *ms2_end, *ms2_loopn;
  const double *pp7_start, *pp7_end, *pp7_loopn;
} or_construct;

/* SumofSquaresFunction_TranscriptionCycleMCMC(construct, data, x) for one cell (tci_oracle.c),
 * with a scratch buffer of at least N + 8 points (oracle_scratch_new). Returns 0 or < 0. */
void *oracle_scratch_new(int64_t cap);
void oracle_scratch_free(void *w);
int oracle_ss_one(const or_construct *cs, const double *t, const double *y1, const double *y2, int64_t N,
                  const double *th, void *w, double *ss_out);

#endif /* TCI_ORACLE_H_ */
