// Host-sanitizer harness for the native CPU helpers.
//
// data_helpers.cpp and dedup.cpp are compiled with -DEMA_EMBEDDED, which turns
// their pybind11 modules into embedded ones, and linked into THIS executable
// together with libpython.  Built with -fsanitize=address,undefined (or
// -fsanitize=thread for the MinHash thread pool) the sanitizer runtime is part
// of the executable itself, so no LD_PRELOAD is needed to load an instrumented
// extension into an uninstrumented python.  The executable runs a python
// script (argv[1]) that imports the embedded `_helpers` / `_dedup` modules and
// drives them; any sanitizer report aborts with a non-zero exit status.
#include <pybind11/embed.h>

#include <cstdio>
#include <string>
#include <vector>

namespace py = pybind11;

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s script.py [args...]\n", argv[0]);
    return 2;
  }
  py::scoped_interpreter guard{};
  try {
    py::list sargv;
    for (int i = 1; i < argc; ++i) sargv.append(std::string(argv[i]));
    py::module_::import("sys").attr("argv") = sargv;
    py::module_::import("runpy").attr("run_path")(std::string(argv[1]),
                                                  py::arg("run_name") = "__main__");
  } catch (py::error_already_set& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
