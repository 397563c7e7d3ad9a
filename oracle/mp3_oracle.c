/*
 * mp3_oracle.c -- TEST INFRASTRUCTURE: CPU restatement of llehouerou/go-mp3.
 *
 * Parity oracle and CPU baseline for the MI355X granule-decode path.  Never
 * linked into the product.  Every section cites the reference file:line it
 * restates (paths relative to the reference repository root).
 *
 * Build (oracle/Makefile):  gcc -O2 -ffp-contract=off -fno-fast-math
 *   -- float32 ops round individually, as gc emits them on linux/amd64
 *   (GOAMD64=v1: no FMA fusion).  Requantization runs in double.
 *
 * PCM parity: UNPINNED by reference golden vectors (none exist, SURVEY.md
 * 8c).  Pinned properties: see mp3_oracle.h.
 */
#include "mp3_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* -ffp-contract=off is mandatory (Makefile) */

#include "huffman_codes.inc"

/* ======================================================================
 * Constant tables
 * ====================================================================== */

/* Scale-factor band boundaries [lsf][sfreq index][long/short]
 * (internal/consts/consts.go:68-97; the "Layer" comments there are the
 * sampling-frequency index, see frame.go:176-182). ISO 11172-3 / 13818-3. */
static const int SFB_LONG[2][3][23] = {
    {{0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 52, 62, 74, 90, 110, 134, 162, 196, 238, 288, 342, 418, 576},
     {0, 4, 8, 12, 16, 20, 24, 30, 36, 42, 50, 60, 72, 88, 106, 128, 156, 190, 230, 276, 330, 384, 576},
     {0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 54, 66, 82, 102, 126, 156, 194, 240, 296, 364, 448, 550, 576}},
    {{0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576},
     {0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 114, 136, 162, 194, 232, 278, 332, 394, 464, 540, 576},
     {0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576}}};
static const int SFB_SHORT[2][3][14] = {
    {{0, 4, 8, 12, 16, 22, 30, 40, 52, 66, 84, 106, 136, 192},
     {0, 4, 8, 12, 16, 22, 28, 38, 50, 64, 80, 100, 126, 192},
     {0, 4, 8, 12, 16, 22, 30, 42, 58, 78, 104, 138, 180, 192}},
    {{0, 4, 8, 12, 18, 24, 32, 42, 56, 74, 100, 132, 174, 192},
     {0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 136, 180, 192},
     {0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 134, 174, 192}}};

/* pretab (frame.go:33), ISO 11172-3 Table B.6 */
static const double PRETAB[22] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 3, 2, 0};
/* intensity-stereo tan table (frame.go:304-306), float32 literals */
static const float IS_RATIOS[6] = {0.000000f, 0.267949f, 0.577350f, 1.000000f, 1.732051f, 3.732051f};
/* antialias butterflies (frame.go:422-425), float32 literals */
static const float AA_CS[8] = {0.857493f, 0.881742f, 0.949629f, 0.983315f,
                               0.995518f, 0.999161f, 0.999899f, 0.999993f};
static const float AA_CA[8] = {-0.514496f, -0.471732f, -0.313377f, -0.181913f,
                               -0.094574f, -0.040966f, -0.014199f, -0.003700f};
/* synthesis window D[i] (frame.go:499-628), ISO 11172-3 Table B.3 */
static const float SYNTH_D[512] = {
    0.000000000f, -0.000015259f, -0.000015259f, -0.000015259f, -0.000015259f, -0.000015259f,
    -0.000015259f, -0.000030518f, -0.000030518f, -0.000030518f, -0.000030518f, -0.000045776f,
    -0.000045776f, -0.000061035f, -0.000061035f, -0.000076294f, -0.000076294f, -0.000091553f,
    -0.000106812f, -0.000106812f, -0.000122070f, -0.000137329f, -0.000152588f, -0.000167847f,
    -0.000198364f, -0.000213623f, -0.000244141f, -0.000259399f, -0.000289917f, -0.000320435f,
    -0.000366211f, -0.000396729f, -0.000442505f, -0.000473022f, -0.000534058f, -0.000579834f,
    -0.000625610f, -0.000686646f, -0.000747681f, -0.000808716f, -0.000885010f, -0.000961304f,
    -0.001037598f, -0.001113892f, -0.001205444f, -0.001296997f, -0.001388550f, -0.001480103f,
    -0.001586914f, -0.001693726f, -0.001785278f, -0.001907349f, -0.002014160f, -0.002120972f,
    -0.002243042f, -0.002349854f, -0.002456665f, -0.002578735f, -0.002685547f, -0.002792358f,
    -0.002899170f, -0.002990723f, -0.003082275f, -0.003173828f, 0.003250122f, 0.003326416f,
    0.003387451f, 0.003433228f, 0.003463745f, 0.003479004f, 0.003479004f, 0.003463745f,
    0.003417969f, 0.003372192f, 0.003280640f, 0.003173828f, 0.003051758f, 0.002883911f,
    0.002700806f, 0.002487183f, 0.002227783f, 0.001937866f, 0.001617432f, 0.001266479f,
    0.000869751f, 0.000442505f, -0.000030518f, -0.000549316f, -0.001098633f, -0.001693726f,
    -0.002334595f, -0.003005981f, -0.003723145f, -0.004486084f, -0.005294800f, -0.006118774f,
    -0.007003784f, -0.007919312f, -0.008865356f, -0.009841919f, -0.010848999f, -0.011886597f,
    -0.012939453f, -0.014022827f, -0.015121460f, -0.016235352f, -0.017349243f, -0.018463135f,
    -0.019577026f, -0.020690918f, -0.021789551f, -0.022857666f, -0.023910522f, -0.024932861f,
    -0.025909424f, -0.026840210f, -0.027725220f, -0.028533936f, -0.029281616f, -0.029937744f,
    -0.030532837f, -0.031005859f, -0.031387329f, -0.031661987f, -0.031814575f, -0.031845093f,
    -0.031738281f, -0.031478882f, 0.031082153f, 0.030517578f, 0.029785156f, 0.028884888f,
    0.027801514f, 0.026535034f, 0.025085449f, 0.023422241f, 0.021575928f, 0.019531250f,
    0.017257690f, 0.014801025f, 0.012115479f, 0.009231567f, 0.006134033f, 0.002822876f,
    -0.000686646f, -0.004394531f, -0.008316040f, -0.012420654f, -0.016708374f, -0.021179199f,
    -0.025817871f, -0.030609131f, -0.035552979f, -0.040634155f, -0.045837402f, -0.051132202f,
    -0.056533813f, -0.061996460f, -0.067520142f, -0.073059082f, -0.078628540f, -0.084182739f,
    -0.089706421f, -0.095169067f, -0.100540161f, -0.105819702f, -0.110946655f, -0.115921021f,
    -0.120697021f, -0.125259399f, -0.129562378f, -0.133590698f, -0.137298584f, -0.140670776f,
    -0.143676758f, -0.146255493f, -0.148422241f, -0.150115967f, -0.151306152f, -0.151962280f,
    -0.152069092f, -0.151596069f, -0.150497437f, -0.148773193f, -0.146362305f, -0.143264771f,
    -0.139450073f, -0.134887695f, -0.129577637f, -0.123474121f, -0.116577148f, -0.108856201f,
    0.100311279f, 0.090927124f, 0.080688477f, 0.069595337f, 0.057617188f, 0.044784546f,
    0.031082153f, 0.016510010f, 0.001068115f, -0.015228271f, -0.032379150f, -0.050354004f,
    -0.069168091f, -0.088775635f, -0.109161377f, -0.130310059f, -0.152206421f, -0.174789429f,
    -0.198059082f, -0.221984863f, -0.246505737f, -0.271591187f, -0.297210693f, -0.323318481f,
    -0.349868774f, -0.376800537f, -0.404083252f, -0.431655884f, -0.459472656f, -0.487472534f,
    -0.515609741f, -0.543823242f, -0.572036743f, -0.600219727f, -0.628295898f, -0.656219482f,
    -0.683914185f, -0.711318970f, -0.738372803f, -0.765029907f, -0.791213989f, -0.816864014f,
    -0.841949463f, -0.866363525f, -0.890090942f, -0.913055420f, -0.935195923f, -0.956481934f,
    -0.976852417f, -0.996246338f, -1.014617920f, -1.031936646f, -1.048156738f, -1.063217163f,
    -1.077117920f, -1.089782715f, -1.101211548f, -1.111373901f, -1.120223999f, -1.127746582f,
    -1.133926392f, -1.138763428f, -1.142211914f, -1.144287109f, 1.144989014f, 1.144287109f,
    1.142211914f, 1.138763428f, 1.133926392f, 1.127746582f, 1.120223999f, 1.111373901f,
    1.101211548f, 1.089782715f, 1.077117920f, 1.063217163f, 1.048156738f, 1.031936646f,
    1.014617920f, 0.996246338f, 0.976852417f, 0.956481934f, 0.935195923f, 0.913055420f,
    0.890090942f, 0.866363525f, 0.841949463f, 0.816864014f, 0.791213989f, 0.765029907f,
    0.738372803f, 0.711318970f, 0.683914185f, 0.656219482f, 0.628295898f, 0.600219727f,
    0.572036743f, 0.543823242f, 0.515609741f, 0.487472534f, 0.459472656f, 0.431655884f,
    0.404083252f, 0.376800537f, 0.349868774f, 0.323318481f, 0.297210693f, 0.271591187f,
    0.246505737f, 0.221984863f, 0.198059082f, 0.174789429f, 0.152206421f, 0.130310059f,
    0.109161377f, 0.088775635f, 0.069168091f, 0.050354004f, 0.032379150f, 0.015228271f,
    -0.001068115f, -0.016510010f, -0.031082153f, -0.044784546f, -0.057617188f, -0.069595337f,
    -0.080688477f, -0.090927124f, 0.100311279f, 0.108856201f, 0.116577148f, 0.123474121f,
    0.129577637f, 0.134887695f, 0.139450073f, 0.143264771f, 0.146362305f, 0.148773193f,
    0.150497437f, 0.151596069f, 0.152069092f, 0.151962280f, 0.151306152f, 0.150115967f,
    0.148422241f, 0.146255493f, 0.143676758f, 0.140670776f, 0.137298584f, 0.133590698f,
    0.129562378f, 0.125259399f, 0.120697021f, 0.115921021f, 0.110946655f, 0.105819702f,
    0.100540161f, 0.095169067f, 0.089706421f, 0.084182739f, 0.078628540f, 0.073059082f,
    0.067520142f, 0.061996460f, 0.056533813f, 0.051132202f, 0.045837402f, 0.040634155f,
    0.035552979f, 0.030609131f, 0.025817871f, 0.021179199f, 0.016708374f, 0.012420654f,
    0.008316040f, 0.004394531f, 0.000686646f, -0.002822876f, -0.006134033f, -0.009231567f,
    -0.012115479f, -0.014801025f, -0.017257690f, -0.019531250f, -0.021575928f, -0.023422241f,
    -0.025085449f, -0.026535034f, -0.027801514f, -0.028884888f, -0.029785156f, -0.030517578f,
    0.031082153f, 0.031478882f, 0.031738281f, 0.031845093f, 0.031814575f, 0.031661987f,
    0.031387329f, 0.031005859f, 0.030532837f, 0.029937744f, 0.029281616f, 0.028533936f,
    0.027725220f, 0.026840210f, 0.025909424f, 0.024932861f, 0.023910522f, 0.022857666f,
    0.021789551f, 0.020690918f, 0.019577026f, 0.018463135f, 0.017349243f, 0.016235352f,
    0.015121460f, 0.014022827f, 0.012939453f, 0.011886597f, 0.010848999f, 0.009841919f,
    0.008865356f, 0.007919312f, 0.007003784f, 0.006118774f, 0.005294800f, 0.004486084f,
    0.003723145f, 0.003005981f, 0.002334595f, 0.001693726f, 0.001098633f, 0.000549316f,
    0.000030518f, -0.000442505f, -0.000869751f, -0.001266479f, -0.001617432f, -0.001937866f,
    -0.002227783f, -0.002487183f, -0.002700806f, -0.002883911f, -0.003051758f, -0.003173828f,
    -0.003280640f, -0.003372192f, -0.003417969f, -0.003463745f, -0.003479004f, -0.003479004f,
    -0.003463745f, -0.003433228f, -0.003387451f, -0.003326416f, 0.003250122f, 0.003173828f,
    0.003082275f, 0.002990723f, 0.002899170f, 0.002792358f, 0.002685547f, 0.002578735f,
    0.002456665f, 0.002349854f, 0.002243042f, 0.002120972f, 0.002014160f, 0.001907349f,
    0.001785278f, 0.001693726f, 0.001586914f, 0.001480103f, 0.001388550f, 0.001296997f,
    0.001205444f, 0.001113892f, 0.001037598f, 0.000961304f, 0.000885010f, 0.000808716f,
    0.000747681f, 0.000686646f, 0.000625610f, 0.000579834f, 0.000534058f, 0.000473022f,
    0.000442505f, 0.000396729f, 0.000366211f, 0.000320435f, 0.000289917f, 0.000259399f,
    0.000244141f, 0.000213623f, 0.000198364f, 0.000167847f, 0.000152588f, 0.000137329f,
    0.000122070f, 0.000106812f, 0.000106812f, 0.000091553f, 0.000076294f, 0.000076294f,
    0.000061035f, 0.000061035f, 0.000045776f, 0.000045776f, 0.000030518f, 0.000030518f,
    0.000030518f, 0.000030518f, 0.000015259f, 0.000015259f, 0.000015259f, 0.000015259f,
    0.000015259f, 0.000015259f};

/* Correctly-rounded float64 values of Go's exactly-folded untyped constants
 * pi/36, pi/12, pi/24 (= pi/(2*12)), pi/72 (= pi/(2*36)), pi/64 and 4/3
 * (imdct.go:25-76, frame.go:38, :494). C's M_PI/12 is 1 ulp off. */
static const double PI_36 = 0x1.657184ae74487p-4;
static const double PI_12 = 0x1.0c152382d7366p-2;
static const double PI_24 = 0x1.0c152382d7366p-3;
static const double PI_72 = 0x1.657184ae74487p-5;
static const double PI_64 = 0x1.921fb54442d18p-5;
static const double FOUR_THIRDS = 0x1.5555555555555p+0;

static float T_NWIN[64][32];   /* synthNWin, frame.go:488-497 */
static float T_WIN[4][36];     /* imdctWinData, imdct.go:21-57 */
static float T_COS12[6][12];   /* cosN12, imdct.go:59-68 */
static float T_COS36[18][36];  /* cosN36, imdct.go:70-79 */
static double T_POW34[8207];   /* powtab34, frame.go:31-40 */
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* Huffman trees rebuilt from the codeword lists (node < 0: leaf). */
#define HT_MAX_NODES 1024
typedef struct { int child[HT_MAX_NODES][2]; int leaf_xy[HT_MAX_NODES]; int n; } htree;
static htree g_trees[34];

static void init_trees(void) {
  for (int t = 0; t < 34; t++) {
    g_trees[t].n = 1;
    g_trees[t].child[0][0] = g_trees[t].child[0][1] = 0;
    g_trees[t].leaf_xy[0] = -1;
  }
  for (int k = 0; k < HUFF_N_CODES; k++) {
    const huff_code_t* c = &HUFF_CODES[k];
    htree* tr = &g_trees[c->tree];
    int node = 0;
    for (int b = c->len - 1; b >= 0; b--) {
      int bit = (c->code >> b) & 1;
      if (tr->child[node][bit] == 0) {
        int nn = tr->n++;
        tr->child[nn][0] = tr->child[nn][1] = 0;
        tr->leaf_xy[nn] = -1;
        tr->child[node][bit] = nn;
      }
      node = tr->child[node][bit];
    }
    tr->leaf_xy[node] = (c->x << 4) | c->y;
  }
}

static void init_tables(void) {
  for (int i = 0; i < 36; i++) T_WIN[0][i] = (float)sin(PI_36 * ((double)i + 0.5));
  for (int i = 0; i < 18; i++) T_WIN[1][i] = (float)sin(PI_36 * ((double)i + 0.5));
  for (int i = 18; i < 24; i++) T_WIN[1][i] = 1.0f;
  for (int i = 24; i < 30; i++) T_WIN[1][i] = (float)sin(PI_12 * ((double)i + 0.5 - 18.0));
  for (int i = 30; i < 36; i++) T_WIN[1][i] = 0.0f;
  for (int i = 0; i < 12; i++) T_WIN[2][i] = (float)sin(PI_12 * ((double)i + 0.5));
  for (int i = 12; i < 36; i++) T_WIN[2][i] = 0.0f;
  for (int i = 0; i < 6; i++) T_WIN[3][i] = 0.0f;
  for (int i = 6; i < 12; i++) T_WIN[3][i] = (float)sin(PI_12 * ((double)i + 0.5 - 6.0));
  for (int i = 12; i < 18; i++) T_WIN[3][i] = 1.0f;
  for (int i = 18; i < 36; i++) T_WIN[3][i] = (float)sin(PI_36 * ((double)i + 0.5));
  for (int i = 0; i < 6; i++)
    for (int j = 0; j < 12; j++)
      T_COS12[i][j] = (float)cos(PI_24 * (2.0 * j + 1.0 + 6.0) * (2.0 * i + 1.0));
  for (int i = 0; i < 18; i++)
    for (int j = 0; j < 36; j++)
      T_COS36[i][j] = (float)cos(PI_72 * (2.0 * j + 1.0 + 18.0) * (2.0 * i + 1.0));
  for (int i = 0; i < 64; i++)
    for (int j = 0; j < 32; j++) T_NWIN[i][j] = (float)cos((double)((16 + i) * (2 * j + 1)) * PI_64);
  for (int i = 0; i < 8207; i++) T_POW34[i] = pow((double)i, FOUR_THIRDS);
  init_trees();
}
static void ensure_init(void) { pthread_once(&g_once, init_tables); }

void orc_tables(float nwin[64][32], float d[512], float win[4][36], float c12[6][12],
                float c36[18][36], double* pow34) {
  ensure_init();
  memcpy(nwin, T_NWIN, sizeof T_NWIN);
  memcpy(d, SYNTH_D, sizeof SYNTH_D);
  memcpy(win, T_WIN, sizeof T_WIN);
  memcpy(c12, T_COS12, sizeof T_COS12);
  memcpy(c36, T_COS36, sizeof T_COS36);
  memcpy(pow34, T_POW34, sizeof T_POW34);
}

/* ======================================================================
 * Bit reader -- internal/bits/bits.go:22-94
 * ====================================================================== */
typedef struct {
  uint8_t* vec;
  long len;
  long byte_pos;
  int bit_pos;
  int err;
} bitrd;

static bitrd* bits_new(uint8_t* vec, long len) { /* takes ownership of vec */
  bitrd* b = (bitrd*)calloc(1, sizeof *b);
  b->vec = vec;
  b->len = len;
  return b;
}
static void bits_free(bitrd* b) {
  if (b) { free(b->vec); free(b); }
}
static int bits_bit(bitrd* b) { /* bits.go:45-56 */
  if (b->len <= b->byte_pos) { b->err = 1; return 0; }
  unsigned v = ((unsigned)b->vec[b->byte_pos] >> (7 - b->bit_pos)) & 1u;
  b->byte_pos += (b->bit_pos + 1) >> 3;
  b->bit_pos = (b->bit_pos + 1) & 7;
  return (int)v;
}
static int bits_bits(bitrd* b, int num) { /* bits.go:58-77 */
  if (num == 0) return 0;
  long cur = b->byte_pos * 8 + b->bit_pos;
  if (cur + num > b->len * 8) { b->err = 1; return 0; }
  uint8_t w[4] = {0, 0, 0, 0};
  for (int k = 0; k < 4 && b->byte_pos + k < b->len; k++) w[k] = b->vec[b->byte_pos + k];
  uint32_t t = ((uint32_t)w[0] << 24) | ((uint32_t)w[1] << 16) | ((uint32_t)w[2] << 8) | w[3];
  t <<= (unsigned)b->bit_pos;
  t >>= (32u - (unsigned)num);
  b->byte_pos += (b->bit_pos + num) >> 3;
  b->bit_pos = (b->bit_pos + num) & 7;
  return (int)t;
}
static long bits_pos(const bitrd* b) { return b->byte_pos * 8 + b->bit_pos; }
static void bits_setpos(bitrd* b, long p) { b->byte_pos = p >> 3; b->bit_pos = (int)(p & 7); }

int orc_bits_read(const uint8_t* data, size_t len, const int* nums, int n, int* out, int* err) {
  uint8_t* v = (uint8_t*)malloc(len ? len : 1);
  memcpy(v, data, len);
  bitrd* b = bits_new(v, (long)len);
  for (int i = 0; i < n; i++) out[i] = nums[i] < 0 ? bits_bit(b) : bits_bits(b, nums[i]);
  *err = b->err;
  bits_free(b);
  return 0;
}

/* ======================================================================
 * Frame header -- internal/frameheader/frameheader.go
 * ====================================================================== */
static int fh_id(uint32_t h) { return (int)((h & 0x00180000u) >> 19); }
static int fh_layer(uint32_t h) { return (int)((h & 0x00060000u) >> 17); }
static int fh_protection(uint32_t h) { return (int)((h & 0x00010000u) >> 16); }
static int fh_bitrate_index(uint32_t h) { return (int)((h & 0x0000f000u) >> 12); }
static int fh_sfreq(uint32_t h) { return (int)((h & 0x00000c00u) >> 10); }
static int fh_padding(uint32_t h) { return (int)((h & 0x00000200u) >> 9); }
static int fh_mode(uint32_t h) { return (int)((h & 0x000000c0u) >> 6); }
static int fh_mode_ext(uint32_t h) { return (int)((h & 0x00000030u) >> 4); }
static int fh_emphasis(uint32_t h) { return (int)(h & 3u); }
static int fh_lsf(uint32_t h) { return fh_id(h) == 3 ? 0 : 1; }             /* :372-378 */
static int fh_granules(uint32_t h) { return 2 >> fh_lsf(h); }               /* :384-387 */
static int fh_bytes_per_frame(uint32_t h) { return 576 * fh_granules(h) * 4; } /* :380-382 */
static int fh_nch(uint32_t h) { return fh_mode(h) == 3 ? 1 : 2; }           /* :503-508 */
static int fh_ms(uint32_t h) { return fh_mode(h) == 1 && (fh_mode_ext(h) & 2); } /* :341-347 */
static int fh_is(uint32_t h) { return fh_mode(h) == 1 && (fh_mode_ext(h) & 1); } /* :349-355 */
static int fh_sample_rate(uint32_t h) {                                     /* :304-318 */
  int lsf = fh_lsf(h);
  switch (fh_sfreq(h)) {
    case 0: return 44100 >> lsf;
    case 1: return 48000 >> lsf;
    case 2: return 32000 >> lsf;
  }
  return 0;
}
static int fh_valid(uint32_t h) {                                           /* :168-189 */
  if ((h & 0xffe00000u) != 0xffe00000u) return 0;
  if (fh_id(h) == 1) return 0;
  if (fh_bitrate_index(h) == 15) return 0;
  if (fh_sfreq(h) == 3) return 0;
  if (fh_layer(h) != 1) return 0;
  if (fh_emphasis(h) == 2) return 0;
  return 1;
}
static int fh_bitrate(uint32_t h) {                                         /* :191-221, ISO tables */
  static const int BR[2][3][16] = {
      {{0, 32000, 40000, 48000, 56000, 64000, 80000, 96000, 112000, 128000, 160000, 192000, 224000, 256000, 320000, 0},
       {0, 32000, 48000, 56000, 64000, 80000, 96000, 112000, 128000, 160000, 192000, 224000, 256000, 320000, 384000, 0},
       {0, 32000, 64000, 96000, 128000, 160000, 192000, 224000, 256000, 288000, 320000, 352000, 384000, 416000, 448000, 0}},
      {{0, 8000, 16000, 24000, 32000, 40000, 48000, 56000, 64000, 80000, 96000, 112000, 128000, 144000, 160000, 0},
       {0, 8000, 16000, 24000, 32000, 40000, 48000, 56000, 64000, 80000, 96000, 112000, 128000, 144000, 160000, 0},
       {0, 32000, 48000, 56000, 64000, 80000, 96000, 112000, 128000, 144000, 160000, 176000, 192000, 224000, 256000, 0}}};
  int layer = fh_layer(h);
  if (layer < 1) return 0;
  return BR[fh_lsf(h)][layer - 1][fh_bitrate_index(h)];
}
static int fh_frame_size(uint32_t h) {                                      /* :223-232 */
  int f = fh_sample_rate(h);
  if (f == 0) return -1;
  return ((144 * fh_bitrate(h)) / f + fh_padding(h)) >> fh_lsf(h);
}
static int fh_side_info_size(uint32_t h) {                                  /* :234-251 */
  int mono = fh_mode(h) == 3;
  if (fh_lsf(h) == 1) return mono ? 9 : 17;
  return mono ? 17 : 32;
}

int orc_header_info(uint32_t h, int* valid, int* spf, int* fsize, int* bpf, int* sr, int64_t* dur) {
  *valid = fh_valid(h);
  *spf = 576 * fh_granules(h);
  *fsize = fh_frame_size(h);
  *bpf = fh_bytes_per_frame(h);
  *sr = fh_sample_rate(h);
  *dur = *sr ? (int64_t)1000000000 * (int64_t)(*spf) / (int64_t)(*sr) : 0; /* :396-403 */
  return 0;
}

/* ======================================================================
 * Byte source -- source.go:22-122 over an in-memory reader
 * (bytes.Reader semantics; `seekable` = implements io.Seeker)
 * ====================================================================== */
typedef struct {
  const uint8_t* data;
  long len;
  long rpos;       /* reader position */
  int seekable;
  uint8_t unread[16];
  int n_unread;
  long pos;        /* source.pos */
} source_t;

/* source.ReadFull (source.go:99-122). Returns bytes read, sets *eof. */
static long src_read_full(source_t* s, uint8_t* buf, long n, int* eof) {
  long got = 0;
  *eof = 0;
  if (s->n_unread > 0) {
    long k = n < s->n_unread ? n : s->n_unread;
    memcpy(buf, s->unread, (size_t)k);
    memmove(s->unread, s->unread + k, (size_t)(s->n_unread - k));
    s->n_unread -= (int)k;
    got = k;
    if (got == n) return got;
  }
  long avail = s->len - s->rpos;
  if (avail < 0) avail = 0;
  long want = n - got;
  long k = want < avail ? want : avail;
  if (k > 0) memcpy(buf + got, s->data + s->rpos, (size_t)k);
  s->rpos += k;
  s->pos += k;
  if (k < want) *eof = 1; /* io.ReadFull: EOF / ErrUnexpectedEOF -> EOF */
  return got + k;
}
static void src_unread(source_t* s, const uint8_t* b, int n) { /* source.go:94-97 */
  memmove(s->unread + n, s->unread, (size_t)s->n_unread);
  memcpy(s->unread, b, (size_t)n);
  s->n_unread += n;
  s->pos -= n;
}
/* source.Seek (source.go:28-40) over bytes.Reader.Seek. 0 ok, -1 error. */
static int src_seek(source_t* s, long off, int whence, long* res) {
  if (!s->seekable) return -1;
  s->n_unread = 0;
  long abs;
  if (whence == 0) abs = off;
  else if (whence == 1) abs = s->rpos + off;
  else abs = s->len + off;
  if (abs < 0) return -1;
  s->rpos = abs;
  s->pos = abs;
  if (res) *res = abs;
  return 0;
}
/* source.skipTags (source.go:42-83). Returns ORC_OK / ORC_EOF / ORC_ERR. */
static int src_skip_tags(source_t* s) {
  for (;;) {
    uint8_t b3[3];
    int eof;
    long n = src_read_full(s, b3, 3, &eof);
    if (eof) return ORC_EOF; /* any error (n<3) is returned as-is: io.EOF */
    (void)n;
    if (memcmp(b3, "TAG", 3) == 0) {
      uint8_t tmp[125];
      src_read_full(s, tmp, 125, &eof);
      if (eof) return ORC_EOF;
    } else if (memcmp(b3, "ID3", 3) == 0) {
      uint8_t tmp[4];
      src_read_full(s, tmp, 3, &eof);
      if (eof) return ORC_EOF;
      n = src_read_full(s, tmp, 4, &eof);
      if (eof) return ORC_EOF;
      if (n != 4) return ORC_OK;
      long size = ((long)tmp[0] << 21) | ((long)tmp[1] << 14) | ((long)tmp[2] << 7) | (long)tmp[3];
      uint8_t* skip = (uint8_t*)malloc((size_t)(size ? size : 1));
      src_read_full(s, skip, size, &eof);
      free(skip);
      if (eof && size > 0) return ORC_EOF;
    } else {
      src_unread(s, b3, 3);
      return ORC_OK;
    }
  }
}

/* frameheader.Read (frameheader.go:279-328). Returns ORC_OK/ORC_EOF/ORC_ERR;
 * *pos_io = position where the header starts. */
static int read_header(source_t* s, long* pos_io, uint32_t* out) {
  uint8_t b[4];
  int eof;
  long n = src_read_full(s, b, 4, &eof);
  if (n < 4) return ORC_EOF; /* n==0: io.EOF; else UnexpectedEOF -> mapped to EOF */
  uint32_t h = ((uint32_t)b[0] << 24) | ((uint32_t)b[1] << 16) | ((uint32_t)b[2] << 8) | b[3];
  long searched = 4;
  long position = *pos_io;
  while (!fh_valid(h)) {
    if (searched >= 64 * 1024) return ORC_EOF; /* SyncSearchLimitError -> EOF (decode.go:59-61) */
    uint8_t c;
    src_read_full(s, &c, 1, &eof);
    if (eof) return ORC_EOF; /* UnexpectedEOF */
    h = (h << 8) | c;
    position++;
    searched++;
  }
  if (fh_bitrate_index(h) == 0) return ORC_ERR; /* free format */
  *pos_io = position;
  *out = h;
  return ORC_OK;
}

/* ======================================================================
 * Side info -- internal/sideinfo/sideinfo.go:33-156
 * ====================================================================== */
typedef struct {
  int main_data_begin, private_bits;
  int scfsi[2][4];
  int part2_3_length[2][2], big_values[2][2], global_gain[2][2], scalefac_compress[2][2];
  int win_switch_flag[2][2], block_type[2][2], mixed_block_flag[2][2];
  int table_select[2][2][3], subblock_gain[2][2][3];
  int region0_count[2][2], region1_count[2][2];
  int preflag[2][2], scalefac_scale[2][2], count1_table_select[2][2], count1[2][2];
} sideinfo_t;

static int read_side_info(source_t* s, uint32_t h, sideinfo_t* si) {
  static const int BITS_TO_READ[2][4] = {{9, 5, 3, 4}, {8, 1, 2, 9}};
  int nch = fh_nch(h);
  int fsize = fh_frame_size(h);
  if (fsize < 0) return ORC_ERR;
  if (fsize > 2000) return ORC_ERR;
  int size = fh_side_info_size(h);
  uint8_t* buf = (uint8_t*)malloc((size_t)size);
  int eof;
  long n = src_read_full(s, buf, size, &eof);
  if (n < size) { free(buf); return eof ? ORC_EOF : ORC_ERR; }
  bitrd* b = bits_new(buf, size);
  int lsf = fh_lsf(h);
  const int* btr = BITS_TO_READ[lsf];
  memset(si, 0, sizeof *si);
  si->main_data_begin = bits_bits(b, btr[0]);
  si->private_bits = bits_bits(b, fh_mode(h) == 3 ? btr[1] : btr[2]);
  if (!lsf)
    for (int ch = 0; ch < nch; ch++)
      for (int k = 0; k < 4; k++) si->scfsi[ch][k] = bits_bits(b, 1);
  for (int gr = 0; gr < fh_granules(h); gr++) {
    for (int ch = 0; ch < nch; ch++) {
      si->part2_3_length[gr][ch] = bits_bits(b, 12);
      si->big_values[gr][ch] = bits_bits(b, 9);
      si->global_gain[gr][ch] = bits_bits(b, 8);
      si->scalefac_compress[gr][ch] = bits_bits(b, btr[3]);
      si->win_switch_flag[gr][ch] = bits_bits(b, 1);
      if (si->win_switch_flag[gr][ch] == 1) {
        si->block_type[gr][ch] = bits_bits(b, 2);
        si->mixed_block_flag[gr][ch] = bits_bits(b, 1);
        for (int r = 0; r < 2; r++) si->table_select[gr][ch][r] = bits_bits(b, 5);
        for (int w = 0; w < 3; w++) si->subblock_gain[gr][ch][w] = bits_bits(b, 3);
        si->region0_count[gr][ch] =
            (si->block_type[gr][ch] == 2 && si->mixed_block_flag[gr][ch] == 0) ? 8 : 7;
        si->region1_count[gr][ch] = 20 - si->region0_count[gr][ch];
      } else {
        for (int r = 0; r < 3; r++) si->table_select[gr][ch][r] = bits_bits(b, 5);
        si->region0_count[gr][ch] = bits_bits(b, 4);
        si->region1_count[gr][ch] = bits_bits(b, 3);
        si->block_type[gr][ch] = 0;
        if (lsf) si->mixed_block_flag[0][ch] = 0;
      }
      if (!lsf) si->preflag[gr][ch] = bits_bits(b, 1);
      si->scalefac_scale[gr][ch] = bits_bits(b, 1);
      si->count1_table_select[gr][ch] = bits_bits(b, 1);
    }
  }
  bits_free(b);
  return ORC_OK;
}

/* ======================================================================
 * Main data -- internal/maindata/maindata.go, huffman.go;
 *              internal/huffman/huffman.go:348-419
 * ====================================================================== */
typedef struct {
  int scalefac_l[2][2][22];
  int scalefac_s[2][2][13][3];
  float is[2][2][576];
} maindata_t;

/* huffman.Decode: bit-serial walk; returns 0 ok, -1 error. */
static int huff_decode(bitrd* m, int table, int* x, int* y, int* v, int* w) {
  *x = *y = *v = *w = 0;
  int tree = HUFF_TABLE_TREE[table];
  int linbits = HUFF_TABLE_LINBITS[table];
  if (tree < 0) return 0; /* empty tables 0, 4, 14 */
  const htree* tr = &g_trees[tree];
  int node = 0, bitsleft = 32;
  while (tr->leaf_xy[node] < 0) {
    node = tr->child[node][bits_bit(m)];
    if (--bitsleft <= 0 || node == 0) return -1;
  }
  *x = (tr->leaf_xy[node] >> 4) & 15;
  *y = tr->leaf_xy[node] & 15;
  if (table > 31) { /* count1 quadruples */
    int q = *y;
    *v = (q >> 3) & 1; *w = (q >> 2) & 1; *x = (q >> 1) & 1; *y = q & 1;
    if (*v && bits_bit(m) == 1) *v = -*v;
    if (*w && bits_bit(m) == 1) *w = -*w;
    if (*x && bits_bit(m) == 1) *x = -*x;
    if (*y && bits_bit(m) == 1) *y = -*y;
  } else {
    if (linbits && *x == 15) *x += bits_bits(m, linbits);
    if (*x && bits_bit(m) == 1) *x = -*x;
    if (linbits && *y == 15) *y += bits_bits(m, linbits);
    if (*y && bits_bit(m) == 1) *y = -*y;
  }
  return 0;
}

/* readHuffman (maindata/huffman.go:27-138) */
static int read_huffman(bitrd* m, uint32_t h, sideinfo_t* si, maindata_t* md, long part2_start,
                        int gr, int ch) {
  float* is = md->is[gr][ch];
  if (si->part2_3_length[gr][ch] == 0) {
    for (int i = 0; i < 576; i++) is[i] = 0.0f;
    return 0;
  }
  long bit_pos_end = part2_start + si->part2_3_length[gr][ch] - 1;
  int region1_start, region2_start;
  if (si->win_switch_flag[gr][ch] == 1 && si->block_type[gr][ch] == 2) {
    region1_start = 36;
    region2_start = 576;
  } else {
    const int* l = SFB_LONG[fh_lsf(h)][fh_sfreq(h)];
    int i = si->region0_count[gr][ch] + 1;
    if (i < 0 || 23 <= i) return -1;
    region1_start = l[i];
    int j = si->region0_count[gr][ch] + si->region1_count[gr][ch] + 2;
    if (j < 0) return -1;
    region2_start = j >= 23 ? 576 : l[j];
  }
  for (int pos = 0; pos < si->big_values[gr][ch] * 2; pos++) {
    if (pos >= 576) return -1; /* #22 */
    int table = pos < region1_start ? si->table_select[gr][ch][0]
                : pos < region2_start ? si->table_select[gr][ch][1]
                                      : si->table_select[gr][ch][2];
    int x, y, v, w;
    if (huff_decode(m, table, &x, &y, &v, &w)) return -1;
    is[pos] = (float)x;
    pos++;
    is[pos] = (float)y;
  }
  int table = si->count1_table_select[gr][ch] + 32;
  int pos = si->big_values[gr][ch] * 2;
  while (pos <= 572 && bits_pos(m) <= bit_pos_end) {
    int x, y, v, w;
    if (huff_decode(m, table, &x, &y, &v, &w)) return -1;
    is[pos++] = (float)v;
    if (pos >= 576) break;
    is[pos++] = (float)w;
    if (pos >= 576) break;
    is[pos++] = (float)x;
    if (pos >= 576) break;
    is[pos++] = (float)y;
  }
  if (bits_pos(m) > bit_pos_end + 1) pos -= 4;
  if (pos < 0) pos = 0;
  si->count1[gr][ch] = pos;
  for (; pos < 576; pos++) is[pos] = 0.0f;
  bits_setpos(m, bit_pos_end + 1);
  return 0;
}

static const int SLEN_MPEG1[16][2] = {{0, 0}, {0, 1}, {0, 2}, {0, 3}, {3, 0}, {1, 1}, {1, 2}, {1, 3},
                                      {2, 1}, {2, 2}, {2, 3}, {3, 1}, {3, 2}, {3, 3}, {4, 2}, {4, 3}};
/* nr_of_sfb (ISO 13818-3 Table 6, as used at maindata.go:44-50) [block][row][part] */
static const int NSFB_MPEG2[3][6][4] = {
    {{6, 5, 5, 5}, {6, 5, 7, 3}, {11, 10, 0, 0}, {7, 7, 7, 0}, {6, 6, 6, 3}, {8, 8, 5, 0}},
    {{9, 9, 9, 9}, {9, 9, 12, 6}, {18, 18, 0, 0}, {12, 12, 12, 0}, {12, 9, 9, 6}, {15, 12, 9, 0}},
    {{6, 9, 9, 9}, {6, 9, 12, 6}, {15, 18, 0, 0}, {6, 15, 12, 0}, {6, 12, 9, 6}, {6, 18, 9, 0}}};
static int g_slen2[512];
static pthread_once_t g_slen_once = PTHREAD_ONCE_INIT;
static void init_slen2(void) { /* maindata.go:52-81: packed slen words */
  for (int a = 0; a < 4; a++)
    for (int b = 0; b < 3; b++) g_slen2[500 + b + 3 * a] = a | (b << 3) | (2 << 12) | (1 << 15);
  for (int a = 0; a < 5; a++)
    for (int b = 0; b < 5; b++)
      for (int c = 0; c < 4; c++)
        for (int d = 0; d < 4; d++) g_slen2[d + 4 * c + 16 * b + 80 * a] = a | (b << 3) | (c << 6) | (d << 9);
  for (int a = 0; a < 5; a++)
    for (int b = 0; b < 5; b++)
      for (int c = 0; c < 4; c++) g_slen2[400 + c + 4 * b + 20 * a] = a | (b << 3) | (c << 6) | (1 << 12);
}

/* getScaleFactorsMpeg2 (maindata.go:119-188). ORC_ERR_PANIC for mixed blocks. */
static int scale_factors_mpeg2(bitrd* m, uint32_t h, sideinfo_t* si, maindata_t* md) {
  pthread_once(&g_slen_once, init_slen2);
  int nch = fh_nch(h);
  memset(md->scalefac_l, 0, sizeof md->scalefac_l);
  memset(md->scalefac_s, 0, sizeof md->scalefac_s);
  for (int ch = 0; ch < nch; ch++) {
    long part2_start = bits_pos(m);
    int slen = g_slen2[si->scalefac_compress[0][ch]];
    si->preflag[0][ch] = (slen >> 15) & 1;
    int blk = 0;
    if (si->block_type[0][ch] == 2) {
      blk++;
      if (si->mixed_block_flag[0][ch] != 0) blk++;
    }
    int sf[64], nsf = 0;
    int row = (slen >> 12) & 7;
    for (int part = 0; part < 4; part++) {
      int nbits = slen & 7;
      slen >>= 3;
      for (int k = 0; k < NSFB_MPEG2[blk][row][part]; k++) sf[nsf++] = nbits > 0 ? bits_bits(m, nbits) : 0;
    }
    for (int k = 0; k < (blk << 1) + 1; k++) sf[nsf++] = 0;
    if (nsf == 22) {
      for (int i = 0; i < 22; i++) md->scalefac_l[0][ch][i] = sf[i];
    } else {
      if (nsf < 39) return ORC_ERR_PANIC; /* index out of range in the reference */
      for (int x = 0; x < 13; x++)
        for (int w = 0; w < 3; w++) md->scalefac_s[0][ch][x][w] = sf[3 * x + w];
    }
    if (read_huffman(m, h, si, md, part2_start, 0, ch)) return ORC_ERR;
  }
  return ORC_OK;
}

/* getScaleFactorsMpeg1 (maindata.go:190-288) */
static int scale_factors_mpeg1(bitrd* m, uint32_t h, sideinfo_t* si, maindata_t* md) {
  int nch = fh_nch(h);
  memset(md->scalefac_l, 0, sizeof md->scalefac_l);
  memset(md->scalefac_s, 0, sizeof md->scalefac_s);
  static const int PART_LO[4] = {0, 6, 11, 16}, PART_HI[4] = {6, 11, 16, 21};
  for (int gr = 0; gr < 2; gr++) {
    for (int ch = 0; ch < nch; ch++) {
      long part2_start = bits_pos(m);
      int slen1 = SLEN_MPEG1[si->scalefac_compress[gr][ch]][0];
      int slen2 = SLEN_MPEG1[si->scalefac_compress[gr][ch]][1];
      if (si->win_switch_flag[gr][ch] == 1 && si->block_type[gr][ch] == 2) {
        if (si->mixed_block_flag[gr][ch] != 0) {
          for (int sfb = 0; sfb < 8; sfb++) md->scalefac_l[gr][ch][sfb] = bits_bits(m, slen1);
          for (int sfb = 3; sfb < 12; sfb++)
            for (int w = 0; w < 3; w++) md->scalefac_s[gr][ch][sfb][w] = bits_bits(m, sfb < 6 ? slen1 : slen2);
        } else {
          for (int sfb = 0; sfb < 12; sfb++)
            for (int w = 0; w < 3; w++) md->scalefac_s[gr][ch][sfb][w] = bits_bits(m, sfb < 6 ? slen1 : slen2);
        }
      } else {
        for (int part = 0; part < 4; part++) {
          int nb = part < 2 ? slen1 : slen2;
          if (si->scfsi[ch][part] == 0 || gr == 0) {
            for (int sfb = PART_LO[part]; sfb < PART_HI[part]; sfb++) md->scalefac_l[gr][ch][sfb] = bits_bits(m, nb);
          } else if (si->scfsi[ch][part] == 1 && gr == 1) {
            for (int sfb = PART_LO[part]; sfb < PART_HI[part]; sfb++)
              md->scalefac_l[1][ch][sfb] = md->scalefac_l[0][ch][sfb];
          }
        }
      }
      if (read_huffman(m, h, si, md, part2_start, gr, ch)) return ORC_ERR;
    }
  }
  return ORC_OK;
}

/* maindata.read: bit reservoir (maindata.go:290-323). Returns new bit reader or NULL. */
static bitrd* reservoir_read(source_t* s, const bitrd* prev, int size, int offset, int* st) {
  if (size > 1500) { *st = ORC_ERR; return NULL; }
  if (size < 0) { *st = ORC_ERR_PANIC; return NULL; } /* make([]byte, <0) panics */
  int eof;
  if (prev && offset > prev->len) { /* underflow quirk: Append(prev, buf), no error */
    uint8_t* buf = (uint8_t*)malloc((size_t)(prev->len + size + 1));
    memcpy(buf, prev->vec, (size_t)prev->len);
    long n = src_read_full(s, buf + prev->len, size, &eof);
    if (n < size) { free(buf); *st = eof ? ORC_EOF : ORC_ERR; return NULL; }
    *st = ORC_OK;
    return bits_new(buf, prev->len + size);
  }
  long keep = prev ? offset : 0;
  uint8_t* buf = (uint8_t*)malloc((size_t)(keep + size + 1));
  if (keep) memcpy(buf, prev->vec + (prev->len - keep), (size_t)keep);
  long n = src_read_full(s, buf + keep, size, &eof);
  if (n < size) { free(buf); *st = eof ? ORC_EOF : ORC_ERR; return NULL; }
  *st = ORC_OK;
  return bits_new(buf, keep + size);
}

/* ======================================================================
 * Frame -- internal/frame/frame.go:42-115
 * ====================================================================== */
typedef struct {
  uint32_t header;
  sideinfo_t si;
  maindata_t* md;   /* shared with the previous frame (reuse, frame.go:98-100) */
  bitrd* mdbits;
  float store[2][32][18];
  float vvec[2][1024];
} frame_t;

static void frame_free(frame_t* f, int free_md) {
  if (!f) return;
  bits_free(f->mdbits);
  if (free_md) free(f->md);
  free(f);
}

/* frame.Read (frame.go:67-115). On success *out = new frame; prev untouched
 * except its MainData which is reused (mutated) like the reference. */
static int frame_read(source_t* s, frame_t* prev, frame_t** out) {
  *out = NULL;
  uint32_t h;
  long pos = s->pos;
  int st = read_header(s, &pos, &h);
  if (st) return st;
  if (fh_protection(h) == 0) {
    uint8_t crc[2];
    int eof;
    long n = src_read_full(s, crc, 2, &eof);
    if (n < 2) return eof ? ORC_EOF : ORC_ERR;
  }
  if (fh_id(h) == 0) return ORC_ERR;    /* MPEG 2.5 */
  if (fh_layer(h) != 1) return ORC_ERR; /* only layer 3 */
  frame_t* f = (frame_t*)calloc(1, sizeof *f);
  f->header = h;
  st = read_side_info(s, h, &f->si);
  if (st) { free(f); return st; }
  /* maindata.Read (maindata.go:85-117) */
  int fsize = fh_frame_size(h);
  if (fsize > 2000) { free(f); return ORC_ERR; }
  int md_size = fsize - fh_side_info_size(h) - 4;
  if (fh_protection(h) == 0) md_size -= 2;
  f->mdbits = reservoir_read(s, prev ? prev->mdbits : NULL, md_size, f->si.main_data_begin, &st);
  if (!f->mdbits) { free(f); return st; }
  f->md = prev ? prev->md : (maindata_t*)calloc(1, sizeof(maindata_t));
  st = fh_lsf(h) ? scale_factors_mpeg2(f->mdbits, h, &f->si, f->md)
                 : scale_factors_mpeg1(f->mdbits, h, &f->si, f->md);
  if (st) {
    bits_free(f->mdbits);
    if (!prev) free(f->md);
    free(f);
    return st;
  }
  if (prev) {
    memcpy(f->store, prev->store, sizeof f->store);
    memcpy(f->vvec, prev->vvec, sizeof f->vvec);
  }
  *out = f;
  return ORC_OK;
}

/* ======================================================================
 * Granule DSP -- frame.go:121-688, imdct.go:83-108
 * One granule, both channels, operating on float Is[2][576] in place.
 * ====================================================================== */
typedef struct {
  int count1, global_gain, scalefac_scale, preflag, win_switch_flag, block_type, mixed_block_flag;
  int subblock_gain[3];
  int scalefac_l[22];
  int scalefac_s[13][3];
} gc_fields;

static int is_short(const gc_fields* c) { return c->win_switch_flag == 1 && c->block_type == 2; }

/* requantizeProcessLong / Short (frame.go:140-174): float64 math, float32 result */
static float requant_long(const gc_fields* c, float x, int sfb) {
  double sf_mult = c->scalefac_scale != 0 ? 1.0 : 0.5;
  double pf = (double)c->preflag * PRETAB[sfb];
  double idx = -(sf_mult * ((double)c->scalefac_l[sfb] + pf)) + 0.25 * ((double)c->global_gain - 210.0);
  double t1 = pow(2.0, idx);
  double t2 = x < 0.0f ? -T_POW34[(int)(-x)] : T_POW34[(int)x];
  return (float)(t1 * t2);
}
static float requant_short(const gc_fields* c, float x, int sfb, int win) {
  double sf_mult = c->scalefac_scale != 0 ? 1.0 : 0.5;
  double idx = -(sf_mult * (double)c->scalefac_s[sfb][win]) +
               0.25 * ((double)c->global_gain - 210.0 - 8.0 * (double)c->subblock_gain[win]);
  double t1 = pow(2.0, idx);
  double t2 = x < 0.0f ? -T_POW34[(int)(-x)] : T_POW34[(int)x];
  return (float)(t1 * t2);
}

/* requantize (frame.go:184-255) */
static void dsp_requantize(const gc_fields* c, const int* sl, const int* ss, float* is) {
  if (is_short(c)) {
    int i = 0, sfb = 0;
    if (c->mixed_block_flag != 0) {
      int next = sl[1];
      for (i = 0; i < 36; i++) {
        if (i == next) { sfb++; next = sl[sfb + 1]; }
        is[i] = requant_long(c, is[i], sfb);
      }
      sfb = 3;
      i = 36;
    }
    int next = ss[sfb + 1] * 3;
    int wl = ss[sfb + 1] - ss[sfb];
    while (i < c->count1) {
      if (i == next) {
        sfb++;
        next = ss[sfb + 1] * 3;
        wl = ss[sfb + 1] - ss[sfb];
      }
      for (int win = 0; win < 3; win++)
        for (int k = 0; k < wl; k++, i++) is[i] = requant_short(c, is[i], sfb, win);
    }
  } else {
    int sfb = 0, next = sl[1];
    for (int i = 0; i < c->count1; i++) {
      if (i == next) { sfb++; next = sl[sfb + 1]; }
      is[i] = requant_long(c, is[i], sfb);
    }
  }
}

/* reorder (frame.go:257-302) */
static void dsp_reorder(const gc_fields* c, const int* ss, float* is) {
  if (!is_short(c)) return;
  float re[576];
  int sfb = c->mixed_block_flag != 0 ? 3 : 0;
  int next = ss[sfb + 1] * 3;
  int wl = ss[sfb + 1] - ss[sfb];
  int i = sfb == 0 ? 0 : 36;
  while (i < 576) {
    if (i == next) {
      int j = 3 * ss[sfb];
      memcpy(&is[j], re, sizeof(float) * (size_t)(3 * wl));
      if (i >= c->count1) return;
      sfb++;
      next = ss[sfb + 1] * 3;
      wl = ss[sfb + 1] - ss[sfb];
    }
    for (int win = 0; win < 3; win++)
      for (int k = 0; k < wl; k++) re[3 * k + win] = is[i++];
  }
  memcpy(&is[3 * ss[12]], re, sizeof(float) * (size_t)(3 * wl));
}

/* stereoProcessIntensityLong / Short (frame.go:308-359) */
static void is_ratios(int pos, float* rl, float* rr) {
  if (pos == 6) { *rl = 1.0f; *rr = 0.0f; return; }
  float r = IS_RATIOS[pos];
  *rl = r / (1.0f + r);
  *rr = 1.0f / (1.0f + r);
}
static void dsp_is_long(const gc_fields* c0, const int* sl, float is[2][576], int sfb) {
  int pos = c0->scalefac_l[sfb];
  if (pos >= 7) return;
  float rl, rr;
  is_ratios(pos, &rl, &rr);
  for (int i = sl[sfb]; i < sl[sfb + 1]; i++) {
    is[0][i] = is[0][i] * rl;
    is[1][i] = is[1][i] * rr;
  }
}
static void dsp_is_short(const gc_fields* c0, const int* ss, float is[2][576], int sfb) {
  int wl = ss[sfb + 1] - ss[sfb];
  for (int win = 0; win < 3; win++) {
    int pos = c0->scalefac_s[sfb][win];
    if (pos >= 7) continue;
    int start = ss[sfb] * 3 + wl * win;
    float rl, rr;
    is_ratios(pos, &rl, &rr);
    for (int i = start; i < start + wl; i++) {
      is[0][i] = is[0][i] * rl;
      is[1][i] = is[1][i] * rr;
    }
  }
}
/* stereo (frame.go:361-420) */
static void dsp_stereo(uint32_t h, const gc_fields c[2], const int* sl, const int* ss, float is[2][576]) {
  if (fh_ms(h)) {
    int max_pos = c[0].count1 > c[1].count1 ? c[0].count1 : c[1].count1;
    const float inv_sqrt2 = 0.70710678118654752440f; /* float32(Sqrt2/2) */
    for (int i = 0; i < max_pos; i++) {
      float l = (is[0][i] + is[1][i]) * inv_sqrt2;
      float r = (is[0][i] - is[1][i]) * inv_sqrt2;
      is[0][i] = l;
      is[1][i] = r;
    }
  }
  if (fh_is(h)) {
    if (is_short(&c[0])) {
      if (c[0].mixed_block_flag != 0) {
        for (int sfb = 0; sfb < 8; sfb++)
          if (sl[sfb] >= c[1].count1) dsp_is_long(&c[0], sl, is, sfb);
        for (int sfb = 3; sfb < 12; sfb++)
          if (ss[sfb] * 3 >= c[1].count1) dsp_is_short(&c[0], ss, is, sfb);
      } else {
        for (int sfb = 0; sfb < 12; sfb++)
          if (ss[sfb] * 3 >= c[1].count1) dsp_is_short(&c[0], ss, is, sfb);
      }
    } else {
      for (int sfb = 0; sfb < 21; sfb++)
        if (sl[sfb] >= c[1].count1) dsp_is_long(&c[0], sl, is, sfb);
    }
  }
}

/* antialias (frame.go:427-452) */
static void dsp_antialias(const gc_fields* c, float* is) {
  if (c->win_switch_flag == 1 && c->block_type == 2 && c->mixed_block_flag == 0) return;
  int sblim = (c->win_switch_flag == 1 && c->block_type == 2 && c->mixed_block_flag == 1) ? 2 : 32;
  for (int sb = 1; sb < sblim; sb++)
    for (int i = 0; i < 8; i++) {
      int li = 18 * sb - 1 - i, ui = 18 * sb + i;
      float lb = is[li] * AA_CS[i] - is[ui] * AA_CA[i];
      float ub = is[ui] * AA_CS[i] + is[li] * AA_CA[i];
      is[li] = lb;
      is[ui] = ub;
    }
}

/* imdct.Win (imdct.go:83-108) */
static void imdct_win(float out[36], const float in[18], int bt) {
  for (int k = 0; k < 36; k++) out[k] = 0.0f;
  if (bt == 2) {
    for (int i = 0; i < 3; i++)
      for (int p = 0; p < 12; p++) {
        float sum = 0.0f;
        for (int m = 0; m < 6; m++) sum = sum + in[i + 3 * m] * T_COS12[m][p];
        out[6 * i + p + 6] = out[6 * i + p + 6] + sum * T_WIN[2][p];
      }
    return;
  }
  for (int p = 0; p < 36; p++) {
    float sum = 0.0f;
    for (int m = 0; m < 18; m++) sum = sum + in[m] * T_COS36[m][p];
    out[p] = sum * T_WIN[bt][p];
  }
}

/* hybridSynthesis + frequencyInversion (frame.go:454-486) */
static void dsp_hybrid(const gc_fields* c, float* is, float store[32][18]) {
  float in[18], raw[36];
  for (int sb = 0; sb < 32; sb++) {
    int bt = c->block_type;
    if (c->win_switch_flag == 1 && c->mixed_block_flag == 1 && sb < 2) bt = 0;
    for (int i = 0; i < 18; i++) in[i] = is[sb * 18 + i];
    imdct_win(raw, in, bt);
    for (int i = 0; i < 18; i++) {
      is[sb * 18 + i] = raw[i] + store[sb][i];
      store[sb][i] = raw[i + 18];
    }
  }
  for (int sb = 1; sb < 32; sb += 2)
    for (int i = 1; i < 18; i += 2) is[sb * 18 + i] = -is[sb * 18 + i];
}

/* Go int(float32) on amd64 (CVTTSS2SQ) then clamp (frame.go:663-669) */
static int16_t pcm_sample(float sum) {
  float t = sum * 32767.0f;
  long long v;
  if (!(t == t) || t >= 9223372036854775808.0f || t < -9223372036854775808.0f)
    v = (long long)0x8000000000000000ull; /* integer indefinite */
  else
    v = (long long)t;
  if (v > 32767) v = 32767;
  else if (v < -32767) v = -32767;
  return (int16_t)v;
}

/* subbandSynthesis (frame.go:630-688); writes stereo-interleaved int16 */
static void dsp_synth(int nch, int ch, const float* is, float* vvec, int16_t* out) {
  float u[512], s[32];
  for (int ss = 0; ss < 18; ss++) {
    memmove(&vvec[64], &vvec[0], sizeof(float) * 960);
    for (int i = 0; i < 32; i++) s[i] = is[i * 18 + ss];
    for (int i = 0; i < 64; i++) {
      float sum = 0.0f;
      for (int j = 0; j < 32; j++) sum = sum + T_NWIN[i][j] * s[j];
      vvec[i] = sum;
    }
    for (int i = 0; i < 512; i += 64) {
      memcpy(&u[i], &vvec[i << 1], sizeof(float) * 32);
      memcpy(&u[i + 32], &vvec[(i << 1) + 96], sizeof(float) * 32);
    }
    for (int i = 0; i < 512; i++) u[i] = u[i] * SYNTH_D[i];
    for (int i = 0; i < 32; i++) {
      float sum = 0.0f;
      for (int j = 0; j < 512; j += 32) sum = sum + u[j + i];
      int16_t smp = pcm_sample(sum);
      int idx = 2 * (32 * ss + i);
      if (nch == 1) { out[idx] = smp; out[idx + 1] = smp; continue; }
      out[idx + ch] = smp;
    }
  }
}

static void granule_dsp(uint32_t h, const gc_fields c[2], float is[2][576], float store[2][32][18],
                        float vvec[2][1024], int16_t* out) {
  const int* sl = SFB_LONG[fh_lsf(h)][fh_sfreq(h)];
  const int* ss = SFB_SHORT[fh_lsf(h)][fh_sfreq(h)];
  int nch = fh_nch(h);
  for (int ch = 0; ch < nch; ch++) {
    dsp_requantize(&c[ch], sl, ss, is[ch]);
    dsp_reorder(&c[ch], ss, is[ch]);
  }
  dsp_stereo(h, c, sl, ss, is);
  for (int ch = 0; ch < nch; ch++) {
    dsp_antialias(&c[ch], is[ch]);
    dsp_hybrid(&c[ch], is[ch], store[ch]);
    dsp_synth(nch, ch, is[ch], vvec[ch], out);
  }
}

static void fields_from_desc(const mp3g_channel* d, gc_fields* c) {
  c->count1 = d->count1;
  c->global_gain = d->global_gain;
  c->scalefac_scale = d->scalefac_scale;
  c->preflag = d->preflag;
  c->win_switch_flag = d->win_switch_flag;
  c->block_type = d->block_type;
  c->mixed_block_flag = d->mixed_block_flag;
  for (int w = 0; w < 3; w++) c->subblock_gain[w] = d->subblock_gain[w];
  for (int k = 0; k < 22; k++) c->scalefac_l[k] = d->scalefac_l[k];
  for (int k = 0; k < 13; k++)
    for (int w = 0; w < 3; w++) c->scalefac_s[k][w] = d->scalefac_s[k][w];
}

static void fields_from_frame(const frame_t* f, int gr, int ch, gc_fields* c) {
  const sideinfo_t* si = &f->si;
  c->count1 = si->count1[gr][ch];
  c->global_gain = si->global_gain[gr][ch];
  c->scalefac_scale = si->scalefac_scale[gr][ch];
  c->preflag = si->preflag[gr][ch];
  c->win_switch_flag = si->win_switch_flag[gr][ch];
  c->block_type = si->block_type[gr][ch];
  c->mixed_block_flag = si->mixed_block_flag[gr][ch];
  for (int w = 0; w < 3; w++) c->subblock_gain[w] = si->subblock_gain[gr][ch][w];
  for (int k = 0; k < 22; k++) c->scalefac_l[k] = f->md->scalefac_l[gr][ch][k];
  for (int k = 0; k < 13; k++)
    for (int w = 0; w < 3; w++) c->scalefac_s[k][w] = f->md->scalefac_s[gr][ch][k][w];
}

static void desc_from_fields(const gc_fields* c, mp3g_channel* d) {
  memset(d, 0, sizeof *d);
  d->count1 = (uint16_t)c->count1;
  d->global_gain = (uint8_t)c->global_gain;
  d->scalefac_scale = (uint8_t)c->scalefac_scale;
  d->preflag = (uint8_t)c->preflag;
  d->win_switch_flag = (uint8_t)c->win_switch_flag;
  d->block_type = (uint8_t)c->block_type;
  d->mixed_block_flag = (uint8_t)c->mixed_block_flag;
  for (int w = 0; w < 3; w++) d->subblock_gain[w] = (uint8_t)c->subblock_gain[w];
  for (int k = 0; k < 22; k++) d->scalefac_l[k] = (uint8_t)c->scalefac_l[k];
  for (int k = 0; k < 13; k++)
    for (int w = 0; w < 3; w++) d->scalefac_s[k][w] = (uint8_t)c->scalefac_s[k][w];
}

/* Frame.Decode (frame.go:121-138): PCM of BytesPerFrame bytes */
static void frame_decode(frame_t* f, int16_t* out) {
  int nch = fh_nch(f->header);
  for (int gr = 0; gr < fh_granules(f->header); gr++) {
    gc_fields c[2];
    memset(c, 0, sizeof c);
    for (int ch = 0; ch < nch; ch++) fields_from_frame(f, gr, ch, &c[ch]);
    granule_dsp(f->header, c, f->md->is[gr], f->store, f->vvec, out + 576 * 2 * gr);
  }
}

void orc_dsp_granules(const mp3g_granule* g, const int16_t* coef, size_t n, mp3g_state* st,
                      int16_t* pcm) {
  ensure_init();
  float is[2][576];
  for (size_t k = 0; k < n; k++) {
    gc_fields c[2];
    memset(c, 0, sizeof c);
    int nch = fh_nch(g[k].header);
    for (int ch = 0; ch < 2; ch++) {
      fields_from_desc(&g[k].ch[ch], &c[ch]);
      for (int i = 0; i < 576; i++) is[ch][i] = (float)coef[k * 1152 + ch * 576 + i];
    }
    (void)nch;
    granule_dsp(g[k].header, c, is, st->store, st->vvec, pcm + k * 1152);
  }
}

int orc_dsp_streams(const mp3g_granule* g, const int16_t* coef, const mp3g_stream* streams,
                    uint32_t n_streams, const mp3g_state* state_in, mp3g_state* state_out,
                    int16_t* pcm) {
  ensure_init();
  mp3g_state st;
  for (uint32_t s = 0; s < n_streams; s++) {
    const mp3g_stream* S = &streams[s];
    if (S->flags & MP3G_STREAM_STATE_IN) st = state_in[s];
    else memset(&st, 0, sizeof st);
    orc_dsp_granules(g + S->first_granule, coef + S->first_granule * 1152, S->n_granules, &st,
                     pcm + S->first_granule * 1152);
    if (S->flags & MP3G_STREAM_STATE_OUT) state_out[s] = st;
  }
  return 0;
}

/* Front end + hybrid synthesis only (frame.go:121-133 up to frequencyInversion,
 * :140-486): writes the float32 lines subbandSynthesis reads, [n][2][576]
 * (mono: [g][1][*] = 0).  State per stream as orc_dsp_streams (store only;
 * vVec is not touched by these stages).  Test-input generator for the
 * standalone polyphase entry point. */
void orc_hybrid_streams(const mp3g_granule* g, const int16_t* coef, const mp3g_stream* streams,
                        uint32_t n_streams, const mp3g_state* state_in, float* is_out) {
  ensure_init();
  static __thread float store[2][32][18]; /* per thread, as orc_synth_streams */
  for (uint32_t s = 0; s < n_streams; s++) {
    const mp3g_stream* S = &streams[s];
    if (S->flags & MP3G_STREAM_STATE_IN) memcpy(store, state_in[s].store, sizeof store);
    else memset(store, 0, sizeof store);
    for (uint64_t k = S->first_granule; k < S->first_granule + S->n_granules; k++) {
      gc_fields c[2];
      float is[2][576];
      memset(c, 0, sizeof c);
      const uint32_t h = g[k].header;
      const int nch = fh_nch(h);
      for (int ch = 0; ch < 2; ch++) {
        fields_from_desc(&g[k].ch[ch], &c[ch]);
        for (int i = 0; i < 576; i++) is[ch][i] = (float)coef[k * 1152 + ch * 576 + i];
      }
      const int* sl = SFB_LONG[fh_lsf(h)][fh_sfreq(h)];
      const int* ss = SFB_SHORT[fh_lsf(h)][fh_sfreq(h)];
      for (int ch = 0; ch < nch; ch++) {
        dsp_requantize(&c[ch], sl, ss, is[ch]);
        dsp_reorder(&c[ch], ss, is[ch]);
      }
      dsp_stereo(h, c, sl, ss, is);
      for (int ch = 0; ch < nch; ch++) {
        dsp_antialias(&c[ch], is[ch]);
        dsp_hybrid(&c[ch], is[ch], store[ch]);
      }
      if (nch == 1) memset(is[1], 0, sizeof is[1]);
      memcpy(is_out + k * 1152, is, sizeof is);
    }
  }
}

/* requantize .. antialias (frame.go:121-131 up to antialias, :140-452): no
 * state crosses granules before the IMDCT, so each granule stands alone. */
void orc_frontend_granules(const mp3g_granule* g, const int16_t* coef, size_t n, float* xr_out) {
  ensure_init();
  for (size_t k = 0; k < n; k++) {
    gc_fields c[2];
    float is[2][576];
    memset(c, 0, sizeof c);
    const uint32_t h = g[k].header;
    const int nch = fh_nch(h);
    for (int ch = 0; ch < 2; ch++) {
      fields_from_desc(&g[k].ch[ch], &c[ch]);
      for (int i = 0; i < 576; i++) is[ch][i] = (float)coef[k * 1152 + ch * 576 + i];
    }
    const int* sl = SFB_LONG[fh_lsf(h)][fh_sfreq(h)];
    const int* ss = SFB_SHORT[fh_lsf(h)][fh_sfreq(h)];
    for (int ch = 0; ch < nch; ch++) {
      dsp_requantize(&c[ch], sl, ss, is[ch]);
      dsp_reorder(&c[ch], ss, is[ch]);
    }
    dsp_stereo(h, c, sl, ss, is);
    for (int ch = 0; ch < nch; ch++) dsp_antialias(&c[ch], is[ch]);
    if (nch == 1) memset(is[1], 0, sizeof is[1]);
    memcpy(xr_out + k * 1152, is, sizeof is);
  }
}

/* subbandSynthesis alone (frame.go:630-688) over streams of granules whose
 * frequency-inverted lines are given as float32 [n][2][576]: the semantics of
 * mp3g_plan_synth_execute.  state: vvec carried per stream (flags as
 * orc_dsp_streams); state_out.store = state_in.store (or zero), untouched. */
int orc_synth_streams(const mp3g_granule* g, const float* is, const mp3g_stream* streams,
                      uint32_t n_streams, const mp3g_state* state_in, mp3g_state* state_out,
                      int16_t* pcm) {
  ensure_init();
  static __thread mp3g_state st; /* per thread: callers may run streams concurrently */
  for (uint32_t s = 0; s < n_streams; s++) {
    const mp3g_stream* S = &streams[s];
    if (S->flags & MP3G_STREAM_STATE_IN) st = state_in[s];
    else memset(&st, 0, sizeof st);
    for (uint64_t k = S->first_granule; k < S->first_granule + S->n_granules; k++) {
      const int nch = fh_nch(g[k].header);
      for (int ch = 0; ch < nch; ch++) dsp_synth(nch, ch, is + k * 1152 + ch * 576, st.vvec[ch], pcm + k * 1152);
    }
    if (S->flags & MP3G_STREAM_STATE_OUT) state_out[s] = st;
  }
  return 0;
}

typedef struct {
  const mp3g_granule* g;
  const int16_t* coef;
  const mp3g_stream* streams;
  uint32_t n_streams;
  int16_t* pcm;
  int tid, nt;
} mt_arg;
static void* mt_worker(void* p) {
  mt_arg* a = (mt_arg*)p;
  mp3g_state* st = (mp3g_state*)malloc(sizeof(mp3g_state));
  for (uint32_t s = (uint32_t)a->tid; s < a->n_streams; s += (uint32_t)a->nt) {
    const mp3g_stream* S = &a->streams[s];
    memset(st, 0, sizeof *st);
    orc_dsp_granules(a->g + S->first_granule, a->coef + S->first_granule * 1152, S->n_granules, st,
                     a->pcm + S->first_granule * 1152);
  }
  free(st);
  return NULL;
}
int orc_dsp_streams_mt(const mp3g_granule* g, const int16_t* coef, const mp3g_stream* streams,
                       uint32_t n_streams, int16_t* pcm, int n_threads) {
  ensure_init();
  if (n_threads < 1) n_threads = 1;
  pthread_t th[256];
  mt_arg args[256];
  if (n_threads > 256) n_threads = 256;
  for (int t = 0; t < n_threads; t++) {
    args[t] = (mt_arg){g, coef, streams, n_streams, pcm, t, n_threads};
    pthread_create(&th[t], NULL, mt_worker, &args[t]);
  }
  for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  return 0;
}

/* ======================================================================
 * Decoder -- decode.go:34-388
 * ====================================================================== */
struct orc_decoder {
  source_t src;
  int sample_rate;
  int64_t length;
  long* frame_starts;
  long n_starts, cap_starts;
  uint8_t* buf;      /* pending PCM */
  long buf_len, buf_off, buf_cap;
  frame_t* frame;
  int64_t pos;
  int64_t bytes_per_frame;
  /* capture */
  int capture;
  mp3g_granule* cap_g;
  int16_t* cap_c;
  size_t cap_n, cap_cap;
};

static void dec_set_frame(orc_decoder* d, frame_t* nf) {
  /* The previous frame's MainData is shared with nf when nf != NULL. */
  if (d->frame) frame_free(d->frame, nf == NULL || nf->md != d->frame->md);
  d->frame = nf;
}

static void capture_frame(orc_decoder* d, const frame_t* f) {
  int ng = fh_granules(f->header), nch = fh_nch(f->header);
  if (d->cap_n + (size_t)ng > d->cap_cap) {
    d->cap_cap = (d->cap_cap + (size_t)ng) * 2;
    d->cap_g = (mp3g_granule*)realloc(d->cap_g, d->cap_cap * sizeof(mp3g_granule));
    d->cap_c = (int16_t*)realloc(d->cap_c, d->cap_cap * 1152 * sizeof(int16_t));
  }
  for (int gr = 0; gr < ng; gr++) {
    mp3g_granule* G = &d->cap_g[d->cap_n];
    int16_t* C = &d->cap_c[d->cap_n * 1152];
    memset(G, 0, sizeof *G);
    memset(C, 0, 1152 * sizeof(int16_t));
    G->header = f->header;
    G->gr = (uint32_t)gr;
    for (int ch = 0; ch < nch; ch++) {
      gc_fields c;
      fields_from_frame(f, gr, ch, &c);
      desc_from_fields(&c, &G->ch[ch]);
      for (int i = 0; i < 576; i++) C[ch * 576 + i] = (int16_t)f->md->is[gr][ch][i];
    }
    d->cap_n++;
  }
}

/* readFrame (decode.go:45-67) */
static int dec_read_frame(orc_decoder* d) {
  frame_t* nf = NULL;
  int st = frame_read(&d->src, d->frame, &nf);
  if (st) {
    dec_set_frame(d, NULL);
    return st; /* EOF-class errors are already mapped to ORC_EOF */
  }
  dec_set_frame(d, nf);
  if (d->capture) capture_frame(d, nf);
  long bpf = fh_bytes_per_frame(nf->header);
  if (d->buf_len + bpf > d->buf_cap) {
    d->buf_cap = (d->buf_len + bpf) * 2;
    d->buf = (uint8_t*)realloc(d->buf, (size_t)d->buf_cap);
  }
  frame_decode(nf, (int16_t*)(d->buf + d->buf_len));
  d->buf_len += bpf;
  return ORC_OK;
}

static void dec_buf_reset(orc_decoder* d) { d->buf_len = 0; d->buf_off = 0; }
static void dec_buf_compact(orc_decoder* d) {
  if (d->buf_off > 0) {
    memmove(d->buf, d->buf + d->buf_off, (size_t)(d->buf_len - d->buf_off));
    d->buf_len -= d->buf_off;
    d->buf_off = 0;
  }
}

/* ensureFrameStartsAndLength (decode.go:154-216) */
static int dec_ensure_length(orc_decoder* d) {
  if (d->length != -1) return ORC_OK;
  if (!d->src.seekable) return ORC_OK;
  long keep = 0;
  src_seek(&d->src, 0, 1, &keep);
  src_seek(&d->src, 0, 0, NULL); /* rewind */
  int st = src_skip_tags(&d->src);
  if (st) return st;
  int64_t l = 0;
  for (;;) {
    uint32_t h;
    long pos = d->src.pos;
    st = read_header(&d->src, &pos, &h);
    if (st == ORC_EOF) break;
    if (st) return st;
    if (d->n_starts == d->cap_starts) {
      d->cap_starts = d->cap_starts ? d->cap_starts * 2 : 1024;
      d->frame_starts = (long*)realloc(d->frame_starts, (size_t)d->cap_starts * sizeof(long));
    }
    d->frame_starts[d->n_starts++] = pos;
    d->bytes_per_frame = fh_bytes_per_frame(h);
    l += d->bytes_per_frame;
    int fsize = fh_frame_size(h);
    src_seek(&d->src, fsize - 4, 1, NULL);
  }
  d->length = l;
  src_seek(&d->src, keep, 0, NULL);
  return ORC_OK;
}

int orc_decoder_new(const uint8_t* data, size_t len, int seekable, orc_decoder** out) {
  ensure_init();
  orc_decoder* d = (orc_decoder*)calloc(1, sizeof *d);
  d->src.data = data;
  d->src.len = (long)len;
  d->src.seekable = seekable;
  d->length = -1;
  int st = src_skip_tags(&d->src);
  if (st == ORC_OK) st = dec_read_frame(d);
  if (st == ORC_OK) {
    d->sample_rate = fh_sample_rate(d->frame->header);
    st = dec_ensure_length(d);
  }
  if (st) { orc_decoder_free(d); *out = NULL; return st; }
  *out = d;
  return ORC_OK;
}

void orc_decoder_free(orc_decoder* d) {
  if (!d) return;
  dec_set_frame(d, NULL);
  free(d->buf);
  free(d->frame_starts);
  free(d->cap_g);
  free(d->cap_c);
  free(d);
}

int orc_decoder_read(orc_decoder* d, uint8_t* out, size_t cap, size_t* n) {
  *n = 0;
  while (d->buf_len - d->buf_off == 0) {
    dec_buf_reset(d);
    int st = dec_read_frame(d);
    if (st) return st;
  }
  long avail = d->buf_len - d->buf_off;
  long k = (long)cap < avail ? (long)cap : avail;
  memcpy(out, d->buf + d->buf_off, (size_t)k);
  d->buf_off += k;
  d->pos += k;
  *n = (size_t)k;
  return ORC_OK;
}

int orc_decoder_seek(orc_decoder* d, int64_t offset, int whence, int64_t* newpos) {
  if (offset == 0 && whence == 1) { *newpos = d->pos; return ORC_OK; }
  int64_t npos;
  switch (whence) {
    case 0: npos = offset; break;
    case 1: npos = d->pos + offset; break;
    case 2: npos = d->length + offset; break;
    default: return ORC_ERR;
  }
  d->pos = npos;
  dec_buf_reset(d);
  dec_set_frame(d, NULL);
  if (d->pos < 0) d->pos = 0;
  if (d->length != -1 && d->pos >= d->length) { *newpos = npos; return ORC_OK; }
  if (d->bytes_per_frame <= 0) return ORC_ERR; /* reference divides by zero */
  int64_t f = d->pos / d->bytes_per_frame;
  if (f > 0) {
    f--;
    if (f >= d->n_starts) return ORC_ERR_PANIC; /* index out of range in the reference */
    if (src_seek(&d->src, d->frame_starts[f], 0, NULL)) return ORC_ERR;
    int st = dec_read_frame(d);
    if (st) return st;
    st = dec_read_frame(d);
    if (st) return st;
    d->buf_off = (long)(d->bytes_per_frame + d->pos % d->bytes_per_frame);
    if (d->buf_off > d->buf_len) { /* slice bounds out of range in the reference */
      dec_buf_reset(d); /* (the process would have ended: leave no negative span for a later Read) */
      return ORC_ERR_PANIC;
    }
  } else {
    if (d->n_starts == 0) return ORC_ERR_PANIC;
    if (src_seek(&d->src, d->frame_starts[0], 0, NULL)) return ORC_ERR;
    int st = dec_read_frame(d);
    if (st) return st;
    d->buf_off = (long)d->pos;
    if (d->buf_off > d->buf_len) {
      dec_buf_reset(d);
      return ORC_ERR_PANIC;
    }
  }
  dec_buf_compact(d);
  *newpos = npos;
  return ORC_OK;
}

int orc_decoder_sample_rate(const orc_decoder* d) { return d->sample_rate; }
int64_t orc_decoder_length(const orc_decoder* d) { return d->length; }
int64_t orc_decoder_bytes_per_frame(const orc_decoder* d) { return d->bytes_per_frame; }
int64_t orc_decoder_pos(const orc_decoder* d) { return d->pos; }
int64_t orc_decoder_n_frames(const orc_decoder* d) { return d->n_starts; }
static int64_t bytes_to_ns(const orc_decoder* d, int64_t b) { /* decode.go:343-348 */
  return (int64_t)1000000000 * b / (int64_t)(d->sample_rate * 4);
}
int64_t orc_decoder_duration_ns(const orc_decoder* d) {
  return d->length == -1 ? -1 : bytes_to_ns(d, d->length);
}
int64_t orc_decoder_position_ns(const orc_decoder* d) { return bytes_to_ns(d, d->pos); }
int orc_decoder_seek_to_time_ns(orc_decoder* d, int64_t t) { /* decode.go:320-341 */
  if (d->length == -1) return ORC_ERR;
  if (t < 0) t = 0;
  int64_t maxd = orc_decoder_duration_ns(d);
  if (t > maxd) t = maxd;
  int64_t b = t * (int64_t)(d->sample_rate * 4) / (int64_t)1000000000;
  b &= ~(int64_t)3;
  int64_t np;
  return orc_decoder_seek(d, b, 0, &np);
}
int orc_decoder_seek_to_sample(orc_decoder* d, int64_t s) { /* decode.go:288-307 */
  if (d->length == -1) return ORC_ERR;
  if (s < 0) s = 0;
  if (s > d->length / 4) s = d->length / 4;
  int64_t np;
  return orc_decoder_seek(d, s * 4, 0, &np);
}

void orc_decoder_capture(orc_decoder* d, int enable) { d->capture = enable; }
size_t orc_decoder_captured(const orc_decoder* d, const mp3g_granule** g, const int16_t** c) {
  *g = d->cap_g;
  *c = d->cap_c;
  return d->cap_n;
}

static int decode_all_impl(const uint8_t* data, size_t len, uint8_t** pcm, size_t* pcm_len,
                           int capture, mp3g_granule** gs, int16_t** cs, size_t* ng) {
  *pcm = NULL;
  *pcm_len = 0;
  orc_decoder* d = NULL;
  ensure_init();
  /* NewDecoder with capture enabled from the first frame */
  d = (orc_decoder*)calloc(1, sizeof *d);
  d->src.data = data;
  d->src.len = (long)len;
  d->src.seekable = 1;
  d->length = -1;
  d->capture = capture;
  int st = src_skip_tags(&d->src);
  if (st == ORC_OK) st = dec_read_frame(d);
  if (st == ORC_OK) {
    d->sample_rate = fh_sample_rate(d->frame->header);
    st = dec_ensure_length(d);
  }
  if (st) { orc_decoder_free(d); return st; }
  size_t cap = 1 << 20, n = 0;
  uint8_t* out = (uint8_t*)malloc(cap);
  for (;;) {
    if (n + 8192 > cap) { cap *= 2; out = (uint8_t*)realloc(out, cap); }
    size_t k;
    st = orc_decoder_read(d, out + n, cap - n, &k);
    if (st) break;
    n += k;
  }
  *pcm = out;
  *pcm_len = n;
  if (capture) {
    *ng = d->cap_n;
    *gs = d->cap_g;
    *cs = d->cap_c;
    d->cap_g = NULL;
    d->cap_c = NULL;
  }
  orc_decoder_free(d);
  return st == ORC_EOF ? ORC_OK : st; /* io.ReadAll treats EOF as success */
}

int orc_decode_all(const uint8_t* data, size_t len, uint8_t** pcm, size_t* pcm_len) {
  return decode_all_impl(data, len, pcm, pcm_len, 0, NULL, NULL, NULL);
}
int orc_decode_all_capture(const uint8_t* data, size_t len, uint8_t** pcm, size_t* pcm_len,
                           mp3g_granule** g, int16_t** c, size_t* n) {
  return decode_all_impl(data, len, pcm, pcm_len, 1, g, c, n);
}
void orc_free(void* p) { free(p); }
