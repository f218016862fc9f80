/* C predict API of mxnet_maintenance_amd (libmxamd_predict.so, built by tools/build_native.py).
 * Same functions and calling conventions as the reference's include/mxnet/c_predict_api.h:
 * every call returns 0 on success and -1 on failure (message from MXGetLastError()); returned
 * pointers stay valid until the next call on the same handle.  dev_type 1 = cpu, 2 = gpu. */
#ifndef MXAMD_C_PREDICT_API_H_
#define MXAMD_C_PREDICT_API_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* PredictorHandle;
typedef void* NDListHandle;

const char* MXGetLastError(void);

int MXPredCreate(const char* symbol_json_str, const void* param_bytes, int param_size, int dev_type, int dev_id,
                 uint32_t num_input_nodes, const char** input_keys, const uint32_t* input_shape_indptr,
                 const uint32_t* input_shape_data, PredictorHandle* out);
int MXPredCreateEx(const char* symbol_json_str, const void* param_bytes, int param_size, int dev_type, int dev_id,
                   const uint32_t num_input_nodes, const char** input_keys, const uint32_t* input_shape_indptr,
                   const uint32_t* input_shape_data, const uint32_t num_provided_arg_dtypes,
                   const char** provided_arg_dtype_names, const int* provided_arg_dtypes, PredictorHandle* out);
int MXPredCreatePartialOut(const char* symbol_json_str, const void* param_bytes, int param_size, int dev_type,
                           int dev_id, uint32_t num_input_nodes, const char** input_keys,
                           const uint32_t* input_shape_indptr, const uint32_t* input_shape_data,
                           uint32_t num_output_nodes, const char** output_keys, PredictorHandle* out);
int MXPredReshape(uint32_t num_input_nodes, const char** input_keys, const uint32_t* input_shape_indptr,
                  const uint32_t* input_shape_data, PredictorHandle handle, PredictorHandle* out);
int MXPredGetOutputShape(PredictorHandle handle, uint32_t index, uint32_t** shape_data, uint32_t* shape_ndim);
int MXPredGetOutputType(PredictorHandle handle, uint32_t index, int* out_dtype);
int MXPredSetInput(PredictorHandle handle, const char* key, const float* data, uint32_t size);
int MXPredForward(PredictorHandle handle);
int MXPredPartialForward(PredictorHandle handle, int step, int* step_left);
int MXPredGetOutput(PredictorHandle handle, uint32_t index, float* data, uint32_t size);
int MXPredFree(PredictorHandle handle);
int MXNDListCreate(const char* nd_file_bytes, int nd_file_size, NDListHandle* out, uint32_t* out_length);
int MXNDListGet(NDListHandle handle, uint32_t index, const char** out_key, const float** out_data,
                const uint32_t** out_shape, uint32_t* out_ndim);
int MXNDListFree(NDListHandle handle);

#ifdef __cplusplus
}
#endif

#endif  /* MXAMD_C_PREDICT_API_H_ */
