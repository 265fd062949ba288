#include "core/process.h"

#include <malloc.h>

#include <cstdlib>
#include <cstring>

#include "core/cpuprof.h"
#include "core/log.h"

namespace bgc {

void tune_malloc() {
  const char* e = std::getenv("BGC_MALLOC_TUNE");
  if (e && std::strcmp(e, "0") == 0) return;
  mallopt(M_TRIM_THRESHOLD, 512 << 20);
  mallopt(M_TOP_PAD, 64 << 20);
  mallopt(M_MMAP_THRESHOLD, 4 << 20);
}

void process_init() {
  tune_malloc();
  log::init_from_env();
  cpuprof::start_from_env();
}

}  // namespace bgc
