/* ref_harness.c -- drives the COMPILED REFERENCE (oracle/_ref/, built by
 * oracle/Makefile from /root/reference/{cg.c,mv_ops.c} where they lie) to
 * produce golden vectors.  TEST INFRASTRUCTURE ONLY.
 *
 * The reference's own main is renamed away (-Dmain=ref_cg_main); this file
 * binds the reference entry points exactly as a caller of cg.c would:
 *   read_input_file  cg.c:23,146   (once per process: static counters, cg.c:235-236)
 *   conj_grad        cg.c:24,88
 *   mv_ops.h:25-42   the op API
 *
 * usage:
 *   ref_harness solve <input.txt> <it0,it1,...>   x after conj_grad(it) as %a
 *   ref_harness ops   <input.txt>                 test_mv_ops' op list (cg.c:368-384)
 *   ref_harness time  <input.txt> <max_iter> <reps>   seconds per conj_grad call
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mv_ops.h"   /* the reference's header, -I/root/reference */

int read_input_file(const char *, struct __mv_sparse *, struct __mv_sparse *);
int conj_grad(int, struct __mv_sparse *, struct __mv_sparse *, struct __mv_sparse **);

static void print_vec(const char *tag, const struct __mv_sparse *v)
{
  printf("%s %d\n", tag, v ? v->size : -1);
  if (!v)
    return;
  for (int i = 0; i < v->size; i++)
    printf("%a\n", v->values[i]);
}

int main(int argc, char **argv)
{
  if (argc < 3) {
    fprintf(stderr, "usage: %s solve|ops|time <input> [args]\n", argv[0]);
    return 2;
  }
  struct __mv_sparse *A = new_mv_struct();
  struct __mv_sparse *b = new_mv_struct();
  if (read_input_file(argv[2], A, b) != 0)
    return 1;

  if (strcmp(argv[1], "solve") == 0 && argc >= 4) {
    char *list = strdup(argv[3]);
    for (char *tok = strtok(list, ","); tok; tok = strtok(NULL, ",")) {
      int it = atoi(tok);
      struct __mv_sparse *x = NULL;
      conj_grad(it, A, b, &x);
      char tag[64];
      snprintf(tag, sizeof tag, "iter %d", it);
      print_vec(tag, x);
    }
    free(list);
  } else if (strcmp(argv[1], "ops") == 0) {
    struct __mv_sparse *r = NULL;
    mv_mult(A, b, &r);
    print_vec("mv_mult", r);
    r = NULL;
    sv_mult(4.0, b, &r);
    print_vec("sv_mult", r);
    printf("dot_product 1\n%a\n", dot_product(b, b));
    r = NULL;
    vec_add(b, b, &r);
    print_vec("vec_add", r);
    r = NULL;
    vec_sub(b, b, &r);
    print_vec("vec_sub", r);
  } else if (strcmp(argv[1], "time") == 0 && argc >= 5) {
    int it = atoi(argv[3]), reps = atoi(argv[4]);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < reps; i++) {
      struct __mv_sparse *x = NULL;
      conj_grad(it, A, b, &x);
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double s = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    printf("%.9f\n", s / reps);
  } else {
    fprintf(stderr, "bad mode\n");
    return 2;
  }
  return 0;
}
