/* oracle/ec_oracle.h -- TEST INFRASTRUCTURE ONLY (see ec_oracle.c header). */
#ifndef EC_ORACLE_H
#define EC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* method ids: src/lio/erasure_tools.h:37-45 */
#define ECO_REED_SOL_VAN   0
#define ECO_REED_SOL_R6_OP 1
#define ECO_CAUCHY_ORIG    2
#define ECO_CAUCHY_GOOD    3
#define ECO_BLAUM_ROTH     4
#define ECO_LIBERATION     5
#define ECO_LIBER8TION     6
#define ECO_RAID4          7

void eco_init(void);
int eco_mul(int a, int b);
int eco_div(int a, int b);
uint32_t eco_mulw(uint32_t a, uint32_t b, int w);   /* w = 8, 16, 32 */
uint32_t eco_invw(uint32_t a, int w);
int eco_coding_matrix(int method, int k, int m, int w, int *out);
int eco_matrix_to_bitmatrix(int k, int m, int w, const int *matrix, int *out);
int eco_generate_plan(long long file_size, int method, int k, int m, int w, int plow, int phigh,
                      int *w_out, int *packet_out, long long *strip_out, int *base_out);
void eco_matrix_encode(int k, int m, int w, const int *matrix, char **data, char **coding, int size);
int eco_bitmatrix_encode(int k, int m, int w, const int *bitmatrix, char **data, char **coding,
                         int size, int packet);
int eco_matrix_decode(int k, int m, int w, const int *matrix, const int *erasures, char **ptrs, int size);
int eco_bitmatrix_decode(int k, int m, int w, const int *bitmatrix, const int *erasures,
                         char **ptrs, int size, int packet);
unsigned int eco_adler32(unsigned int adler, const unsigned char *buf, long long len);

#ifdef __cplusplus
}
#endif
#endif
