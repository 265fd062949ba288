// crdgen: prints the UserBootstrap CustomResourceDefinition as YAML on stdout with no
// extra trailing newline (reference src/crdgen.rs:3-8, `print!("{}", yaml)`).
#include <cstdio>
#include <exception>
#include <string>

#include "crd/schema.h"

int main() {
  try {
    std::string y = bgc::crd::crd_yaml();
    std::fwrite(y.data(), 1, y.size(), stdout);
    return 0;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
}
