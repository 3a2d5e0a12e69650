// Minimal YAML reader for configuration files written by kubectl and friends (kubeconfig), into
// the in-tree Json DOM. Supported: block mappings and sequences (incl. "- key: value" compact
// mappings and sequences indented at their parent key's level), plain / 'single' / "double"
// quoted scalars with null/bool/int/float resolution, one-line flow collections ([a, b], {k: v}),
// literal/folded block scalars (| |- > >-), comments, and "---" (the first document is returned).
// Not supported: anchors/aliases, tags, multi-line plain scalars, complex keys.
#pragma once

#include <stdexcept>
#include <string>

#include "gpupool/json.h"

namespace gpupool {

class YamlError : public std::runtime_error {
 public:
  using std::runtime_error::runtime_error;
};

Json yaml_parse(const std::string& text);  // throws YamlError

}  // namespace gpupool
