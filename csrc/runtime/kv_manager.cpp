// Paged KV-cache block manager (host runtime, C++).
//
// Owns the free list of fixed-size KV pages of ONE rank and the page list of every live
// sequence. The engine calls it once per scheduled sequence per step, so the hot paths
// (append a token slot, build the decode block table / slot / position arrays for a whole
// batch) are O(batch) C++ loops writing straight into caller-provided int32 buffers
// (numpy / pinned torch memory) instead of Python lists.
//
// Pages are reference-counted so a prefix can be shared by forked sequences (parallel
// sampling / beam search); a shared last page is copied-on-write by the caller via the
// `cow` result of append_slot.
#include "kv_manager.h"

#include <pybind11/stl.h>

namespace bfly_rt {

void register_kv_manager(py::module_& m) {
  py::class_<KVBlockManager>(m, "KVBlockManager")
      .def(py::init<int, int>(), py::arg("num_blocks"), py::arg("block_size"))
      .def_property_readonly("num_blocks", &KVBlockManager::num_blocks)
      .def_property_readonly("block_size", &KVBlockManager::block_size)
      .def_property_readonly("num_free", &KVBlockManager::num_free)
      .def_property_readonly("num_seqs", &KVBlockManager::num_seqs)
      .def("has", &KVBlockManager::has)
      .def("blocks_needed", &KVBlockManager::blocks_needed)
      .def("can_allocate", &KVBlockManager::can_allocate)
      .def("allocate", &KVBlockManager::allocate)
      .def("append_slot", &KVBlockManager::append_slot)
      .def("extend", &KVBlockManager::extend)
      .def("extend_blocks", &KVBlockManager::extend_blocks)
      .def("can_append", &KVBlockManager::can_append)
      .def("fork", &KVBlockManager::fork)
      .def("free", &KVBlockManager::free)
      .def("block_table", &KVBlockManager::block_table)
      .def("length", &KVBlockManager::length)
      .def("fill_decode_tables", &KVBlockManager::fill_decode_tables)
      .def_property_readonly("num_cached_blocks", &KVBlockManager::num_cached_blocks)
      .def("block_hashes", &KVBlockManager::block_hashes)
      .def("match_prefix", &KVBlockManager::match_prefix)
      .def("allocate_prefixed", &KVBlockManager::allocate_prefixed)
      .def("register_blocks", &KVBlockManager::register_blocks);
}

}  // namespace bfly_rt
