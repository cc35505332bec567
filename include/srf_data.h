/* srf_data.h -- C ABI of the TF-free host side of the SRF path: the input
 * pipeline and the CTC beam-search decoder (host only).
 *
 * Replaces the TFRecord I/O the reference does through TensorFlow:
 *   tf.data.TFRecordDataset + tf.io.parse_single_example of
 *     {input_speech: VarLen float32, target_label: VarLen int64,
 *      input_length: int64, target_length: int64, utt_id: bytes}
 *   (tfsr/data/load_speech_data.py:43-85), and tf.io.TFRecordWriter +
 *   tf.train.Example serialisation (tfsr/data/save_speech_data.py:119-120,178-186).
 *
 * TFRecord framing: uint64le length, uint32le masked CRC32C(length bytes),
 * data, uint32le masked CRC32C(data); mask(c) = ((c >> 15) | (c << 17)) + 0xa282ead8.
 * Example wire format: tensorflow/core/example/{example,feature}.proto.
 *
 * Return codes: 0 ok, 1 end of file (srf_tfr_next), < 0 error
 * (-1 bad argument / open failure, -5 corrupt record or CRC mismatch,
 *  -6 malformed Example); srf_data_last_error() holds a thread-local message.
 */
#ifndef SRF_DATA_H_
#define SRF_DATA_H_
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

const char* srf_data_last_error(void);

/* CRC-32C (Castagnoli) and the TFRecord mask of it. */
uint32_t srf_crc32c(const void* data, size_t n);
uint32_t srf_crc32c_masked(const void* data, size_t n);

/* One parsed speech Example.  Pointers stay valid until the next
 * srf_tfr_next / srf_tfr_close on the same reader. */
typedef struct {
  const float* input_speech;   /* input_length * feat_dim floats, row-major */
  int64_t n_input_speech;
  const int64_t* target_label;
  int64_t n_target_label;
  int64_t input_length;        /* -1 when absent */
  int64_t target_length;       /* -1 when absent */
  const char* utt_id;          /* not NUL-terminated; NULL when absent */
  int64_t utt_id_len;
} srf_speech_example;

/* verify_crc = 1 checks both CRCs of every record (TFRecordDataset does). */
void* srf_tfr_open(const char* path, int verify_crc);
int srf_tfr_next(void* reader, srf_speech_example* out);
/* Raw record bytes of the last srf_tfr_next (serialized Example). */
const uint8_t* srf_tfr_record(void* reader, size_t* n);
int srf_tfr_close(void* reader);

/* Parse one serialized Example (no framing) with the scratch of a handle from
 * srf_tfr_open or srf_example_parser_new (free it with srf_tfr_close). */
void* srf_example_parser_new(void);
int srf_example_parse(void* handle, const uint8_t* data, size_t n, srf_speech_example* out);

void* srf_tfr_writer_open(const char* path);
/* utt_id may be NULL (field omitted).  Features are written in key order
 * (input_length, input_speech, target_label, target_length, utt_id), which is
 * protobuf's deterministic serialisation of the map. */
int srf_tfr_write_example(void* writer, const float* input_speech, int64_t n_input_speech,
                          const int64_t* target_label, int64_t n_target_label, int64_t input_length,
                          int64_t target_length, const char* utt_id, int64_t utt_id_len);
int srf_tfr_write_record(void* writer, const uint8_t* data, size_t n);
int srf_tfr_writer_close(void* writer);

/* CTC prefix beam search of one utterance, replacing tf.nn.ctc_beam_search_decoder
 * in process_test_step (trainer_sr.py:109-112; top_paths = 1, no re-merge of repeats).
 * logits [T][C] row-major fp32 (a log-softmax is applied per frame), blank index
 * `blank`.  Writes the most probable labelling (at most T labels) to out_labels, its
 * length to *out_len and its log probability to *out_log_prob (may be NULL).
 * Returns 0, or -1 on a bad argument. */
int srf_ctc_beam_search(const float* logits, int T, int C, int blank, int beam_width, int32_t* out_labels,
                        int* out_len, float* out_log_prob);

#ifdef __cplusplus
}
#endif
#endif /* SRF_DATA_H_ */
