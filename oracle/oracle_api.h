// oracle/oracle_api.h — TEST INFRASTRUCTURE ONLY: C entry points of the CPU
// restatement (loaded by tests/ via ctypes).  Layouts mirror cv::KeyPoint
// (28 B) and line_descriptor::KeyLine; they are declared here independently
// of the product headers so the checker shares no code with the product.
#pragma once
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
typedef struct { float x, y, size, angle, response; int32_t octave, class_id; } plvi_keypoint;
#ifdef __cplusplus
}
#endif
