// One-sided peer mailboxes (see mailbox.hip). Registered into bcfl._C by bindings.cpp.
#pragma once
#include <torch/extension.h>

namespace bcfl_comm {
void register_mailbox(pybind11::module& m);
}  // namespace bcfl_comm
