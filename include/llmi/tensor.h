// C++ boundary types with the reference's names and meaning, for callers of
// the llmi C ABI that were written against Mr-wang27/llm-inference:
//   Device / DataType / Tensor / TensorWrapper<T> / TensorMap  (src/utils/tensor.h:13-304)
//   LLM_CHECK / LLM_CHECK_WITH_INFO                              (src/utils/macro.h:113-133)
// Non-owning views over device (or host) pointers, as in the reference
// (TensorWrapper::data is not owned, tensor.h:117-124). Header-only, no HIP types.
#pragma once
#include <cstdint>
#include <functional>
#include <numeric>
#include <sstream>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../llmi.h"

namespace llmi {

// ---- error convention: std::runtime_error("[oneLLM][ERROR] ...") like the reference
inline void check_fail(const char* cond, const std::string& info, const char* file, int line) {
    std::ostringstream os;
    os << "[oneLLM][ERROR] " << (info.empty() ? std::string("Assertion fail: ") + cond : info) << " " << file
       << ":" << line;
    throw std::runtime_error(os.str());
}
// a non-zero llmi_* status becomes the same exception, carrying llmi_last_error()
inline void check_status(int rc, const char* what) {
    if (rc != LLMI_OK) {
        std::ostringstream os;
        os << "[oneLLM][ERROR] " << what << " failed (" << rc << "): " << llmi_last_error();
        throw std::runtime_error(os.str());
    }
}
}  // namespace llmi

#define LLM_CHECK(cond) \
    do { if (!(cond)) ::llmi::check_fail(#cond, "", __FILE__, __LINE__); } while (0)
#define LLM_CHECK_WITH_INFO(cond, info) \
    do { if (!(cond)) ::llmi::check_fail(#cond, (info), __FILE__, __LINE__); } while (0)
#define LLMI_CALL(expr) ::llmi::check_status((expr), #expr)

enum Device { CPU_PINNED, CPU, GPU };
enum DataType { FP32, FP16, INT8, INT32, BOOL, BYTES, UNSUPPORTED };

using half_t = uint16_t;  // fp16 storage type (bits); this API includes no HIP headers

template <typename T> inline DataType getTensorType() {
    if (std::is_same<T, float>::value) return FP32;
    if (std::is_same<T, half_t>::value) return FP16;
    if (std::is_same<T, int>::value) return INT32;
    if (std::is_same<T, int8_t>::value) return INT8;
    if (std::is_same<T, bool>::value) return BOOL;
    if (std::is_same<T, char>::value) return BYTES;
    return UNSUPPORTED;
}
inline int llmiDtype(DataType t) {
    switch (t) {
        case FP32: return LLMI_F32;
        case FP16: return LLMI_F16;
        case INT8: return LLMI_I8;
        case INT32: return LLMI_I32;
        default: return -1;
    }
}

template <typename T> class TensorWrapper;

struct Tensor {
    Device location = GPU;
    DataType dtype = FP32;
    std::vector<int> shape;
    Tensor() = default;
    Tensor(Device loc, DataType dt, std::vector<int> s) : location(loc), dtype(dt), shape(std::move(s)) {}
    virtual ~Tensor() = default;
    virtual int size() const {
        return shape.empty() ? 0 : std::accumulate(shape.begin(), shape.end(), 1, std::multiplies<int>());
    }
    // the reference's as<T>() is an unchecked static_cast (tensor.h:63-66); a view of the
    // wrong element type would be read silently as another type, so it is checked here
    template <typename T> TensorWrapper<T>* as() {
        LLM_CHECK_WITH_INFO(getTensorType<T>() == dtype, "Tensor::as<T>(): the tensor's dtype (" + std::to_string(dtype) +
                                                             ") is not T (" + std::to_string(getTensorType<T>()) + ")");
        return static_cast<TensorWrapper<T>*>(this);
    }
    std::string DeviceString() const { return location == GPU ? "GPU" : location == CPU ? "CPU" : "CPU_PINNED"; }
    virtual std::string toString() const {
        std::ostringstream os;
        os << "Tensor[where=" << DeviceString() << ", type=" << dtype << ", shape=[";
        for (size_t i = 0; i < shape.size(); ++i) os << (i ? ", " : "") << shape[i];
        os << "]]";
        return os.str();
    }
};

template <typename T>
class TensorWrapper : public Tensor {
public:
    T* data = nullptr;  // not owned
    TensorWrapper(Device loc, DataType dt, std::vector<int> s) : Tensor(loc, dt, std::move(s)) {}
    TensorWrapper(Device loc, DataType dt, std::vector<int> s, T* d) : Tensor(loc, dt, std::move(s)), data(d) {
        LLM_CHECK_WITH_INFO(getTensorType<T>() == dt,
                            "when build TensorWrapper, the passed in data type should be same as dtype in params");
    }
    int size() const override { return (data == nullptr) ? 0 : Tensor::size(); }
    T getVal(int id) const {
        LLM_CHECK(location == CPU);  // host tensors only (tensor.h:142-154)
        return data[id];
    }
    T getVal() const { return getVal(0); }
    T* getPtr() const { return data; }
    T* getPtrByOffset(int off) const { return data + off; }
};

struct TensorMap {
    std::unordered_map<std::string, Tensor*> tensor_map_;
    TensorMap() = default;
    TensorMap(std::initializer_list<std::pair<std::string, Tensor*>> init) {
        for (auto& kv : init) {
            LLM_CHECK_WITH_INFO(isValid(kv.second), kv.first + " is not a valid tensor, skipping insert into TensorMap");
            insert(kv.first, kv.second);
        }
    }
    size_t size() const { return tensor_map_.size(); }
    bool isExist(const std::string& k) const { return tensor_map_.count(k) != 0; }
    static bool isValid(const Tensor* t) { return t != nullptr && t->size() > 0; }
    void insert(const std::string& k, Tensor* v) { tensor_map_[k] = v; }
    std::vector<std::string> keys() const {
        std::vector<std::string> out;
        for (auto& kv : tensor_map_) out.push_back(kv.first);
        return out;
    }
    Tensor* at(const std::string& k) {
        if (!isExist(k)) {
            std::string ks;
            for (auto& n : keys()) ks += n + ",";
            LLM_CHECK_WITH_INFO(false, "Cannot find a tensor of name " + k + " in the tensor map (keys: " + ks + ")");
        }
        return tensor_map_.at(k);
    }
    Tensor* operator[](const std::string& k) { return at(k); }
};

using IntDict = std::unordered_map<std::string, int>;     // src/utils/params.h:5
using floatDict = std::unordered_map<std::string, float>;  // src/utils/params.h:6
