/* Test operator for dora-gpu-runtime, written against include/dora_operator_api.h in the style
 * of the reference's C operator example: counts `message` inputs, answers each on `counter`
 * with a text line, echoes the bytes on `echo`, and re-sends any other input's Arrow array
 * unchanged on `same` (the Arrow extension of this build).  Returns DORA_STATUS_STOP on an
 * input `stop`. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dora_gpu.h"
#include "dora_operator_api.h"

DoraInitResult_t dora_init_operator(void) {
  int* counter = (int*)calloc(1, sizeof(int));
  DoraInitResult_t r = {.operator_context = counter};
  return r;
}

DoraResult_t dora_drop_operator(void* operator_context) {
  free(operator_context);
  DoraResult_t r = {0};
  return r;
}

OnEventResult_t dora_on_event(RawEvent_t* event, const SendOutput_t* send_output,
                              void* operator_context) {
  OnEventResult_t result = {.status = DORA_STATUS_CONTINUE};
  int* counter = (int*)operator_context;
  if (event->input != NULL) {
    char* id = dora_read_input_id(event->input);
    if (strcmp(id, "message") == 0) {
      Vec_uint8_t data = dora_read_data(event->input);
      if (data.ptr == NULL) {
        result.result = dora_operator_error("message is not a UInt8 array without nulls");
      } else {
        *counter += 1;
        char line[100];
        int n = snprintf(line, sizeof(line), "The current counter value is %d", *counter);
        result.result = dora_send_operator_output(send_output, "counter", (const uint8_t*)line,
                                                  (size_t)n);
        if (result.result.error == NULL)
          result.result = dora_send_operator_output(send_output, "echo", data.ptr, data.len);
        dora_free_data(data);
      }
    } else if (strcmp(id, "stop") == 0) {
      result.status = DORA_STATUS_STOP;
    } else {
      const struct ArrowArray* a = NULL;
      const struct ArrowSchema* s = NULL;
      if (dora_input_arrow(event->input, &a, &s) == 0) {
        /* the input keeps ownership of its array: hand the runtime a borrowed view (no release
         * callbacks), which it packs into the output sample before this call returns */
        struct ArrowArray view = *a;
        struct ArrowSchema sview = *s;
        view.release = NULL;
        sview.release = NULL;
        result.result = dora_send_operator_output_arrow(send_output, "same", &view, &sview);
      }
    }
    dora_free_input_id(id);
  }
  return result;
}
