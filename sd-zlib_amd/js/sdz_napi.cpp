// sdz_napi.cpp -- thin N-API addon over libsdz.so (include/sdz.h).
//
// This is the binding a maintainer of @stardazed/zlib would add: it exposes the
// batched C ABI to JavaScript with zero-copy input views (napi_get_typedarray_info)
// and outputs written straight into fresh ArrayBuffers.  All API semantics
// (validation, messages, auto-detect) live in index.mjs, which mirrors
// src/sd-inflate.ts and src/sd-deflate.ts.
#include <node_api.h>

#include <cstring>
#include <string>
#include <vector>

#include "sdz.h"

namespace {

#define NAPI_OK(call)                                                   \
    do {                                                                \
        if ((call) != napi_ok) {                                        \
            napi_throw_error(env, nullptr, "sdz addon: N-API call failed"); \
            return nullptr;                                             \
        }                                                               \
    } while (0)

bool get_bytes(napi_env env, napi_value v, const uint8_t** data, size_t* len) {
    bool is_ta = false;
    napi_is_typedarray(env, v, &is_ta);
    if (!is_ta) return false;
    napi_typedarray_type t;
    size_t n = 0, off = 0;
    void* p = nullptr;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &t, &n, &p, &ab, &off) != napi_ok) return false;
    if (t != napi_uint8_array) return false;
    *data = (const uint8_t*)p;
    *len = n;
    return true;
}

void set_int(napi_env env, napi_value o, const char* k, int64_t v) {
    napi_value x;
    napi_create_double(env, (double)v, &x);
    napi_set_named_property(env, o, k, x);
}
void set_str(napi_env env, napi_value o, const char* k, const char* s, size_t n) {
    napi_value x;
    napi_create_string_latin1(env, s, n, &x);
    napi_set_named_property(env, o, k, x);
}
void set_bool(napi_env env, napi_value o, const char* k, bool b) {
    napi_value x;
    napi_get_boolean(env, b, &x);
    napi_set_named_property(env, o, k, x);
}

// devices: an optional array of HIP device ids (sdz_*_batch_multi); false when absent/empty
bool get_devices(napi_env env, size_t argc, napi_value* argv, size_t k, std::vector<int32_t>* devs) {
    if (argc <= k) return false;
    bool is_arr = false;
    napi_is_array(env, argv[k], &is_arr);
    if (!is_arr) return false;
    uint32_t nd = 0;
    napi_get_array_length(env, argv[k], &nd);
    for (uint32_t i = 0; i < nd; ++i) {
        napi_value e;
        int32_t d = 0;
        if (napi_get_element(env, argv[k], i, &e) != napi_ok || napi_get_value_int32(env, e, &d) != napi_ok) return false;
        devs->push_back(d);
    }
    return !devs->empty();
}

// the multi-GPU call's stats as a JS object (gather timed apart from compute)
napi_value stats_object(napi_env env, const sdz_multi_stats& st) {
    napi_value o, ks;
    napi_create_object(env, &o);
    napi_value x;
    napi_create_double(env, st.wall_ms, &x); napi_set_named_property(env, o, "wallMs", x);
    napi_create_double(env, st.compute_ms, &x); napi_set_named_property(env, o, "computeMs", x);
    napi_create_double(env, st.gather_ms, &x); napi_set_named_property(env, o, "gatherMs", x);
    set_bool(env, o, "rccl", st.collective != 0);
    napi_create_array_with_length(env, (size_t)st.nshards, &ks);
    for (int32_t k = 0; k < st.nshards; ++k) {
        napi_value sh;
        napi_create_object(env, &sh);
        set_int(env, sh, "streams", st.streams[k]);
        set_int(env, sh, "bytesIn", (int64_t)st.bytes_in[k]);
        set_int(env, sh, "bytesOut", (int64_t)st.bytes_out[k]);
        napi_create_double(env, st.kernel_ms[k], &x); napi_set_named_property(env, sh, "kernelMs", x);
        napi_set_element(env, ks, (uint32_t)k, sh);
    }
    napi_set_named_property(env, o, "shards", ks);
    return o;
}

const char* verdict(int v) { return v == SDZ_MATCH ? "match" : v == SDZ_MISMATCH ? "mismatch" : "unchecked"; }
const char* status_name(int s) {
    switch (s) {
    case SDZ_OK: return "OK";
    case SDZ_DATA_ERROR: return "DATA_ERROR";
    case SDZ_NEED_DICT: return "NEED_DICT";
    case SDZ_DICT_MISMATCH: return "DICT_MISMATCH";
    case SDZ_TRUNCATED: return "TRUNCATED";
    case SDZ_OUT_OVERFLOW: return "OUT_OVERFLOW";
    case SDZ_TRAILING: return "TRAILING";
    case SDZ_INTERNAL: return "INTERNAL";
    case SDZ_TOO_SMALL: return "TOO_SMALL";
    case SDZ_CARRY_OVERFLOW: return "CARRY_OVERFLOW";
    default: return "BAD_RECORD";
    }
}

// inflateBatch(streams: Uint8Array[], format: number, outCaps: number[], dict: Uint8Array|null,
//              devices?: number[]) -- with devices, LPT shards over those GPUs (result.stats)
napi_value InflateBatch(napi_env env, napi_callback_info info) {
    size_t argc = 5;
    napi_value argv[5];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    uint32_t n = 0;
    NAPI_OK(napi_get_array_length(env, argv[0], &n));
    int32_t fmt = 0;
    NAPI_OK(napi_get_value_int32(env, argv[1], &fmt));
    std::vector<const uint8_t*> in(n);
    std::vector<size_t> in_len(n), cap(n);
    std::vector<uint8_t*> out(n);
    std::vector<napi_value> abs(n);
    for (uint32_t i = 0; i < n; ++i) {
        napi_value e, c;
        NAPI_OK(napi_get_element(env, argv[0], i, &e));
        if (!get_bytes(env, e, &in[i], &in_len[i])) {
            napi_throw_type_error(env, nullptr, "inflateBatch: streams must be Uint8Arrays");
            return nullptr;
        }
        NAPI_OK(napi_get_element(env, argv[2], i, &c));
        double dc = 0;
        NAPI_OK(napi_get_value_double(env, c, &dc));
        cap[i] = (size_t)dc;
        void* p = nullptr;
        NAPI_OK(napi_create_arraybuffer(env, cap[i] ? cap[i] : 1, &p, &abs[i]));
        out[i] = (uint8_t*)p;
    }
    const uint8_t* dict = nullptr;
    size_t dict_len = 0;
    napi_valuetype dt;
    napi_typeof(env, argv[3], &dt);
    if (dt != napi_null && dt != napi_undefined) get_bytes(env, argv[3], &dict, &dict_len);
    std::vector<sdz_inflate_record> rec(n);
    std::vector<int32_t> devs;
    const bool multi = get_devices(env, argc, argv, 4, &devs);
    sdz_multi_stats st;
    int rc = multi ? sdz_inflate_batch_multi(in.data(), in_len.data(), out.data(), cap.data(), rec.data(), n, fmt, dict,
                                             dict_len, devs.data(), (int32_t)devs.size(), &st)
                   : sdz_inflate_batch(in.data(), in_len.data(), out.data(), cap.data(), rec.data(), n, fmt, dict, dict_len);
    if (rc) {
        napi_throw_error(env, nullptr, (std::string("libsdz: ") + sdz_last_error()).c_str());
        return nullptr;
    }
    napi_value arr;
    NAPI_OK(napi_create_array_with_length(env, n, &arr));
    for (uint32_t i = 0; i < n; ++i) {
        const sdz_inflate_record& r = rec[i];
        napi_value o, ta;
        NAPI_OK(napi_create_object(env, &o));
        const char* sn = status_name(r.status);
        set_str(env, o, "status", sn, strlen(sn));
        const char* zm = sdz_zmsg(r.zmsg);
        set_str(env, o, "zmsg", zm, strlen(zm));
        set_bool(env, o, "complete", r.complete);
        set_bool(env, o, "success", r.success);
        set_str(env, o, "checksum", verdict(r.checksum_verdict), strlen(verdict(r.checksum_verdict)));
        set_str(env, o, "fileSize", verdict(r.size_verdict), strlen(verdict(r.size_verdict)));
        if (r.name_len && (size_t)r.name_off + r.name_len <= in_len[i])
            set_str(env, o, "fileName", (const char*)in[i] + r.name_off, r.name_len);
        else
            set_str(env, o, "fileName", "", 0);
        set_int(env, o, "mtime", r.mtime);
        set_int(env, o, "container", r.container);
        size_t len = r.out_len < cap[i] ? (size_t)r.out_len : cap[i];
        NAPI_OK(napi_create_typedarray(env, napi_uint8_array, len, abs[i], 0, &ta));
        napi_set_named_property(env, o, "data", ta);
        NAPI_OK(napi_set_element(env, arr, i, o));
    }
    if (multi) napi_set_named_property(env, arr, "stats", stats_object(env, st));
    return arr;
}

// deflateBatch(streams: Uint8Array[], level, format, fileNameLatin1: Uint8Array, mtime,
//              dict: Uint8Array|null, devices?: number[])
napi_value DeflateBatch(napi_env env, napi_callback_info info) {
    size_t argc = 7;
    napi_value argv[7];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    uint32_t n = 0;
    NAPI_OK(napi_get_array_length(env, argv[0], &n));
    int32_t level = 6, fmt = 1;
    uint32_t mtime = 0;
    NAPI_OK(napi_get_value_int32(env, argv[1], &level));
    NAPI_OK(napi_get_value_int32(env, argv[2], &fmt));
    const uint8_t* fname = nullptr;
    size_t fname_len = 0;
    get_bytes(env, argv[3], &fname, &fname_len);
    double dm = 0;
    NAPI_OK(napi_get_value_double(env, argv[4], &dm));
    mtime = (uint32_t)(int64_t)dm;
    const uint8_t* dict = nullptr;
    size_t dict_len = 0;
    if (argc > 5) {
        napi_valuetype dt;
        napi_typeof(env, argv[5], &dt);
        if (dt != napi_null && dt != napi_undefined) get_bytes(env, argv[5], &dict, &dict_len);
    }
    std::vector<const uint8_t*> in(n);
    std::vector<size_t> in_len(n), cap(n);
    std::vector<uint8_t*> out(n);
    std::vector<napi_value> abs(n);
    for (uint32_t i = 0; i < n; ++i) {
        napi_value e;
        NAPI_OK(napi_get_element(env, argv[0], i, &e));
        if (!get_bytes(env, e, &in[i], &in_len[i])) {
            napi_throw_type_error(env, nullptr, "deflateBatch: streams must be Uint8Arrays");
            return nullptr;
        }
        cap[i] = (size_t)sdz_deflate_bound(in_len[i], fmt, (uint32_t)fname_len);
        void* p = nullptr;
        NAPI_OK(napi_create_arraybuffer(env, cap[i], &p, &abs[i]));
        out[i] = (uint8_t*)p;
    }
    std::vector<sdz_deflate_record> rec(n);
    std::vector<int32_t> devs;
    const bool multi = get_devices(env, argc, argv, 6, &devs);
    sdz_multi_stats st;
    int rc = multi ? sdz_deflate_batch_multi(in.data(), in_len.data(), out.data(), cap.data(), rec.data(), n, level, fmt,
                                             fname_len ? fname : nullptr, fname_len, mtime, dict, dict_len, devs.data(),
                                             (int32_t)devs.size(), &st)
                   : sdz_deflate_batch(in.data(), in_len.data(), out.data(), cap.data(), rec.data(), n, level, fmt,
                                       fname_len ? fname : nullptr, fname_len, mtime, dict, dict_len);
    if (rc) {
        napi_throw_error(env, nullptr, (std::string("libsdz: ") + sdz_last_error()).c_str());
        return nullptr;
    }
    napi_value arr;
    NAPI_OK(napi_create_array_with_length(env, n, &arr));
    for (uint32_t i = 0; i < n; ++i) {
        napi_value o, ta;
        NAPI_OK(napi_create_object(env, &o));
        const char* sn = status_name(rec[i].status);
        set_str(env, o, "status", sn, strlen(sn));
        set_int(env, o, "checksum", rec[i].checksum);
        size_t len = rec[i].out_len < cap[i] ? (size_t)rec[i].out_len : cap[i];
        NAPI_OK(napi_create_typedarray(env, napi_uint8_array, len, abs[i], 0, &ta));
        napi_set_named_property(env, o, "data", ta);
        NAPI_OK(napi_set_element(env, arr, i, o));
    }
    if (multi) napi_set_named_property(env, arr, "stats", stats_object(env, st));
    return arr;
}

// ---- one incremental Inflater (sdz_inflater_*): state stays on the device between appends

void inflater_finalize(napi_env, void* data, void*) { sdz_inflater_destroy((sdz_inflater*)data); }

// inflaterCreate(raw: boolean, dict: Uint8Array|null) -> handle
napi_value InflaterCreate(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    bool raw = false;
    NAPI_OK(napi_get_value_bool(env, argv[0], &raw));
    const uint8_t* dict = nullptr;
    size_t dict_len = 0;
    napi_valuetype dt;
    napi_typeof(env, argv[1], &dt);
    if (dt != napi_null && dt != napi_undefined) get_bytes(env, argv[1], &dict, &dict_len);
    sdz_inflater* z = sdz_inflater_create(raw ? SDZ_FMT_RAW : SDZ_FMT_CONTAINER, dict, dict_len);
    if (!z) {
        napi_throw_error(env, nullptr, (std::string("libsdz: ") + sdz_last_error()).c_str());
        return nullptr;
    }
    napi_value h;
    NAPI_OK(napi_create_external(env, z, inflater_finalize, nullptr, &h));
    return h;
}

// inflaterAppend(handle, chunk: Uint8Array) -> { status, zmsg, complete, success, checksum,
// fileSize, nameOff, nameLen, mtime, container, data }
napi_value InflaterAppend(napi_env env, napi_callback_info info) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    void* hp = nullptr;
    NAPI_OK(napi_get_value_external(env, argv[0], &hp));
    const uint8_t* in = nullptr;
    size_t len = 0;
    if (!get_bytes(env, argv[1], &in, &len)) {
        napi_throw_type_error(env, nullptr, "data must be an ArrayBuffer or buffer view");
        return nullptr;
    }
    const uint8_t* out = nullptr;
    size_t out_len = 0;
    sdz_inflate_record r;
    if (sdz_inflater_append((sdz_inflater*)hp, in, len, &out, &out_len, &r)) {
        napi_throw_error(env, nullptr, (std::string("libsdz: ") + sdz_last_error()).c_str());
        return nullptr;
    }
    napi_value o, ab, ta;
    NAPI_OK(napi_create_object(env, &o));
    const char* sn = status_name(r.status);
    set_str(env, o, "status", sn, strlen(sn));
    const char* zm = sdz_zmsg(r.zmsg);
    set_str(env, o, "zmsg", zm, strlen(zm));
    set_bool(env, o, "complete", r.complete);
    set_bool(env, o, "success", r.success);
    set_str(env, o, "checksum", verdict(r.checksum_verdict), strlen(verdict(r.checksum_verdict)));
    set_str(env, o, "fileSize", verdict(r.size_verdict), strlen(verdict(r.size_verdict)));
    set_int(env, o, "nameOff", r.name_off);
    set_int(env, o, "nameLen", r.name_len);
    set_int(env, o, "mtime", r.mtime);
    set_int(env, o, "container", r.container);
    void* p = nullptr;
    NAPI_OK(napi_create_arraybuffer(env, out_len ? out_len : 1, &p, &ab));
    if (out_len) memcpy(p, out, out_len);
    NAPI_OK(napi_create_typedarray(env, napi_uint8_array, out_len, ab, 0, &ta));
    napi_set_named_property(env, o, "data", ta);
    return o;
}

// ---- one incremental Deflater (sdz_deflater_*): compressor state stays on the device

void deflater_finalize(napi_env, void* data, void*) { sdz_deflater_destroy((sdz_deflater*)data); }

// deflaterCreate(level, format (0 raw, 1 deflate, 2 gzip), fileNameLatin1: Uint8Array, mtime,
// dict: Uint8Array|null) -> handle
napi_value DeflaterCreate(napi_env env, napi_callback_info info) {
    size_t argc = 5;
    napi_value argv[5];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    int32_t level = 6, fmt = 1;
    uint32_t mtime = 0;
    NAPI_OK(napi_get_value_int32(env, argv[0], &level));
    NAPI_OK(napi_get_value_int32(env, argv[1], &fmt));
    const uint8_t* fname = nullptr;
    size_t fname_len = 0;
    get_bytes(env, argv[2], &fname, &fname_len);
    NAPI_OK(napi_get_value_uint32(env, argv[3], &mtime));
    const uint8_t* dict = nullptr;
    size_t dict_len = 0;
    napi_valuetype dt;
    napi_typeof(env, argv[4], &dt);
    if (dt != napi_null && dt != napi_undefined) get_bytes(env, argv[4], &dict, &dict_len);
    sdz_deflater* z = sdz_deflater_create(level, fmt, fname, fname_len, mtime,
                                          dt != napi_null && dt != napi_undefined ? (dict ? dict : (const uint8_t*)"") : nullptr,
                                          dict_len);
    if (!z) {
        napi_throw_error(env, nullptr, (std::string("libsdz: ") + sdz_last_error()).c_str());
        return nullptr;
    }
    napi_value h;
    NAPI_OK(napi_create_external(env, z, deflater_finalize, nullptr, &h));
    return h;
}

// deflaterAppend(handle, chunk: Uint8Array, finish: boolean) -> { status, data }
napi_value DeflaterAppend(napi_env env, napi_callback_info info) {
    size_t argc = 3;
    napi_value argv[3];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    void* hp = nullptr;
    NAPI_OK(napi_get_value_external(env, argv[0], &hp));
    const uint8_t* in = nullptr;
    size_t len = 0;
    if (!get_bytes(env, argv[1], &in, &len)) {
        napi_throw_type_error(env, nullptr, "data must be an ArrayBuffer or buffer view");
        return nullptr;
    }
    bool finish = false;
    NAPI_OK(napi_get_value_bool(env, argv[2], &finish));
    const uint8_t* out = nullptr;
    size_t out_len = 0;
    sdz_deflate_record r;
    if (sdz_deflater_append((sdz_deflater*)hp, in, len, finish ? 1 : 0, &out, &out_len, &r)) {
        napi_throw_error(env, nullptr, (std::string("libsdz: ") + sdz_last_error()).c_str());
        return nullptr;
    }
    napi_value o, ab, ta;
    NAPI_OK(napi_create_object(env, &o));
    const char* sn = status_name(r.status);
    set_str(env, o, "status", sn, strlen(sn));
    void* p = nullptr;
    NAPI_OK(napi_create_arraybuffer(env, out_len ? out_len : 1, &p, &ab));
    if (out_len) memcpy(p, out, out_len);
    NAPI_OK(napi_create_typedarray(env, napi_uint8_array, out_len, ab, 0, &ta));
    napi_set_named_property(env, o, "data", ta);
    return o;
}

napi_value Checksum(napi_env env, napi_callback_info info, bool crc) {
    size_t argc = 2;
    napi_value argv[2];
    NAPI_OK(napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr));
    const uint8_t* p = nullptr;
    size_t n = 0;
    if (!get_bytes(env, argv[0], &p, &n)) {
        napi_throw_type_error(env, nullptr, "source must be a BufferSource");
        return nullptr;
    }
    int32_t seed = 0;
    NAPI_OK(napi_get_value_int32(env, argv[1], &seed));
    int32_t r = 0;
    int rc = crc ? sdz_crc32_checked(p, n, seed, &r) : sdz_adler32_checked(p, n, seed, &r);
    if (rc) {
        napi_throw_error(env, nullptr, (std::string("libsdz: ") + sdz_last_error()).c_str());
        return nullptr;
    }
    napi_value x;
    NAPI_OK(napi_create_int32(env, r, &x));
    return x;
}
napi_value Adler32(napi_env env, napi_callback_info info) { return Checksum(env, info, false); }
napi_value Crc32(napi_env env, napi_callback_info info) { return Checksum(env, info, true); }

napi_value DeviceCount(napi_env env, napi_callback_info) {
    napi_value x;
    napi_create_int32(env, sdz_device_count(), &x);
    return x;
}

napi_value Init(napi_env env, napi_value exports) {
    napi_property_descriptor d[] = {
        { "inflateBatch", nullptr, InflateBatch, nullptr, nullptr, nullptr, napi_enumerable, nullptr },
        { "deflateBatch", nullptr, DeflateBatch, nullptr, nullptr, nullptr, napi_enumerable, nullptr },
        { "adler32", nullptr, Adler32, nullptr, nullptr, nullptr, napi_enumerable, nullptr },
        { "crc32", nullptr, Crc32, nullptr, nullptr, nullptr, napi_enumerable, nullptr },
        { "deviceCount", nullptr, DeviceCount, nullptr, nullptr, nullptr, napi_enumerable, nullptr },
        { "inflaterCreate", nullptr, InflaterCreate, nullptr, nullptr, nullptr, napi_enumerable, nullptr },
        { "inflaterAppend", nullptr, InflaterAppend, nullptr, nullptr, nullptr, napi_enumerable, nullptr },
        { "deflaterCreate", nullptr, DeflaterCreate, nullptr, nullptr, nullptr, napi_enumerable, nullptr },
        { "deflaterAppend", nullptr, DeflaterAppend, nullptr, nullptr, nullptr, napi_enumerable, nullptr },
    };
    napi_define_properties(env, exports, sizeof d / sizeof d[0], d);
    return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
