/* cg_main.c -- drop-in for the reference's CLI (cg.c:42-85):
 *
 *   cg <input-data> <max-iterations> [suppress-output]
 *
 * Same argv, same stdout ("CG took approx %d seconds", then print_sparse of
 * x, mv_ops.c:77-95); the solve runs on the MI355X through libcgx's
 * conj_grad.  Like the reference, the optional third argument is parsed
 * (cg.c:56-57) but does not change the output.  The input is read with
 * cgx_read_input_file (the reference's 4-line format, cg.c:146-218).
 *
 * Environment (read here, not by the library): CGX_MODE=exact -> the
 * reference's sequential dot-product order (bit-identical x), CGX_ALG=cg1 ->
 * Chronopoulos-Gear, CGX_ALG=sr -> the single-reduction recurrence where the
 * matrix takes its one-launch step (HS otherwise), CGX_DEVICE=<ordinal> ->
 * the GPU, CGX_INPUT_CACHE=<path>
 * -> read the input through the binary cache at <path>
 * (cgx_read_input_cached: the text is parsed once per input version). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "cgx.h"

int main(int argc, char **argv)
{
  if (argc < 3) {
    fprintf(stderr, "Usage: %s <input-data> <max-iterations> [suppress-output]\n", argv[0]);
    return -1;
  }
  const char *input_file = argv[1];
  int max_iterations = (int)strtol(argv[2], NULL, 10);
  int no_output = (argc == 4 && argv[3][0] == 'y');
  (void)no_output;

  const char *mode = getenv("CGX_MODE"), *alg = getenv("CGX_ALG"), *dev = getenv("CGX_DEVICE");
  const int exact = mode && strcmp(mode, "exact") == 0;
  int a = CGX_ALG_HS;
  if (!exact && alg && strcmp(alg, "cg1") == 0) a = CGX_ALG_CG1;
  if (!exact && alg && strcmp(alg, "sr") == 0) a = CGX_ALG_SR;
  if (cgx_ops_set_mode(exact ? CGX_MODE_EXACT : CGX_MODE_FAST, a) != 0 ||
      (dev && *dev && cgx_ops_set_device(atoi(dev)) != 0)) {
    fprintf(stderr, "cg: %s\n", cgx_last_error());
    return 1;
  }

  struct __mv_sparse *mat_A = new_mv_struct();
  struct __mv_sparse *vec_b = new_mv_struct();
  struct __mv_sparse *vec_x = NULL;
  const char *cache = getenv("CGX_INPUT_CACHE");
  if ((cache && *cache ? cgx_read_input_cached(input_file, cache, mat_A, vec_b, NULL)
                       : cgx_read_input_file(input_file, mat_A, vec_b)) != 0)
    return -1;

  time_t start = time(NULL);
  int rc = conj_grad(max_iterations, mat_A, vec_b, &vec_x);
  time_t end = time(NULL);
  if (rc != 0) {
    fprintf(stderr, "cg: conj_grad failed (%d): %s\n", rc, cgx_last_error());
    return 1;
  }
  printf("CG took approx %d seconds\n", (int)(end - start));
  print_sparse(vec_x);

  cgx_free_mv_deep(mat_A);
  cgx_free_mv_deep(vec_b);
  cgx_free_mv_deep(vec_x);
  return 0;
}
