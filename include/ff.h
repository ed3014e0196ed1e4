/* Drop-in name for callers that `#include "ff.h"` (the reference wrapper does):
 * the fflib2 subset implemented by libesgd.so. */
#include "esgd_ff.h"
