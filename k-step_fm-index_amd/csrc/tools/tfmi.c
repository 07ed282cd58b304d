/*
 * tfmiBMP / tfmiAC -- offline layout transforms (reference
 * src/transformIndexBitmaps.c:297-333, src/transformIndexAlternateCounters.c:481-527):
 *   tfmiBMP <index.fmi>   -> <index.fmi>.interleaving            (tag 101)
 *   tfmiAC  <index.fmi>   -> <index.fmi>.ac, .interleaving.ac     (tags 200, 201)
 * The mode is taken from the program name (argv[0] ending in "AC") or --ac.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../../../include/kstep_fmi.h"

#define CHECK(e) do { int32_t _e = (e); if (_e) { fprintf(stderr, "%s\n", errorCommon(_e)); return EXIT_FAILURE; } } while (0)

int main(int argc, char *argv[])
{
  void *index = NULL, *a = NULL, *b = NULL;
  size_t l = strlen(argv[0]);
  int ac = (l >= 2 && !strcmp(argv[0] + l - 2, "AC")) || (argc > 2 && !strcmp(argv[2], "--ac"));
  if (argc < 2) { fprintf(stderr, "usage: %s <index.fmi> [--ac]\n", argv[0]); return EXIT_FAILURE; }
  CHECK(kfmi_load_index_tag(argv[1], 100, &index));
  if (ac) {
    CHECK(kfmi_transform_ac(index, &a, &b));
    CHECK(saveIndex(argv[1], a));
    CHECK(saveIndex(argv[1], b));
    freeIndex(&a);
    freeIndex(&b);
  } else {
    CHECK(kfmi_transform_interleave(index, &a));
    CHECK(saveIndex(argv[1], a));
    freeIndex(&a);
  }
  freeIndex(&index);
  return EXIT_SUCCESS;
}
