/* TEST INFRASTRUCTURE ONLY: the in-process JNIEnv of fake_env.c */
#ifndef KHST_TEST_FAKE_ENV_H
#define KHST_TEST_FAKE_ENV_H
#include <stdint.h>

#include "jni.h"

enum { FK_ARRAY = 1, FK_DIRECT, FK_CLASS, FK_STRING, FK_THROWABLE };
typedef struct FakeObj {
  int kind;
  jsize len;  /* arrays: elements */
  int esz;    /* arrays: element bytes */
  void* data; /* arrays: the elements; direct buffers: the address */
  jlong cap;  /* direct buffers */
  char name[128];
  char msg[512];
} FakeObj;
typedef struct {
  int pending;
  char exc_class[128];
  char exc_msg[512];
  int node_missing_calls;
  uint8_t node_missing_hash[32];
  uint64_t region_bytes;
} FakeState;
extern FakeState fake;

JNIEnv* fake_env(void);
FakeObj* fake_array(jsize len, int esz, const void* init);
FakeObj* fake_direct(void* p, jlong cap);
#endif
