// model_file.hpp -- rwkv.cpp model file reader (host side of the load path).
//
// Format: reference docs/FILE_FORMAT.md:10-68, rwkv_file_format.inc:100-316.
// Architecture detection and the per-version parameter table follow
// rwkv_model_loading.inc:128-419.
#pragma once

#include <stdint.h>
#include <string>
#include <unordered_map>
#include <vector>

#include "errors.hpp"

namespace rwkvmi {

struct FileHeader {
    uint32_t magic, version, n_vocab, n_embed, n_layer, data_type;
};

struct HostTensor {
    std::string name;
    uint32_t type = 0, ndim = 0;
    uint32_t ne[3] = {1, 1, 1};
    std::vector<uint8_t> data;
    uint64_t nel() const { return (uint64_t)ne[0] * ne[1] * ne[2]; }
};

struct ModelFile {
    FileHeader header{};
    int arch_major = 4, arch_minor = 0;
    int64_t head_count = 0, head_size = 0;
    std::vector<HostTensor> tensors;
    std::unordered_map<std::string, size_t> index;

    const HostTensor * find(const std::string & name) const {
        auto it = index.find(name);
        return it == index.end() ? nullptr : &tensors[it->second];
    }
};

// bytes of a tensor (rwkv_utilities.inc:1-4); 0 when the type is unsupported
size_t type_nbytes(uint32_t type, uint64_t nel);
size_t type_block_bytes(uint32_t type);
bool type_supported(uint32_t type);
bool type_quantized(uint32_t type);
const char * type_name(uint32_t type);
int type_from_name(const char * name);

// Reads and validates the header (rwkv_file_format.inc:115-142).  Sets global error flags.
bool read_file_header(FILE * f, FileHeader & h);

// Loads the whole file and checks the per-version parameter table.  Sets global error flags
// exactly like rwkv_load_model_from_file (rwkv_model_loading.inc:288-419).
// layer_begin/layer_end: only the data of blocks.<i>.* with i in [layer_begin, layer_end) (plus
// emb.weight / blocks.0.ln0 when layer_begin == 0, ln_out / head when layer_end == n_layer) is
// read; every other tensor keeps its header (all shapes are still checked) and empty data.
bool load_model_file(const char * path, ModelFile & mf, uint32_t layer_begin = 0, uint32_t layer_end = UINT32_MAX);

// fp16 helpers (round-to-nearest-even, same as F16C)
uint16_t f32_to_f16(float f);
float f16_to_f32(uint16_t h);

}  // namespace rwkvmi
