#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static uint32_t head_be(const uint8_t*b,uint32_t p,uint32_t len){uint32_t v=0;for(int k=0;k<4;k++) if(p+k<len) v|=(uint32_t)b[p+k]<<(8*k); return __builtin_bswap32(v);}
/* walk statistics of the k_match kernel for one block */
void stats(const uint8_t* blk, uint32_t len, uint32_t chain, uint32_t nice, double* out)
{
    uint16_t* p4=calloc(len+1,2); int32_t* h4=malloc(65536*4); for(int i=0;i<65536;i++)h4[i]=-1;
    for(uint32_t p=0;p<len;p++){ uint32_t hd=p?head_be(blk,p,len):0; uint32_t a=p?(hd*0x1e35a7bdu)>>16:0; p4[p]=h4[a]<0?0:p-h4[a]; h4[a]=p; }
    uint8_t* W=calloc(len+600,1); memcpy(W,blk,len);
    double hops=0, pass=0, mbytes=0, nicestop=0, full=0;
    for(uint32_t p=0;p<len;p++){ uint32_t cl=2,it=0,d=p4[p],q=p-d;
        for(;;){ if(it>=chain||d==0||p-q>=32768){ if(it>=chain) full++; break;} hops++;
            if(W[q+cl]==W[p+cl]){ pass++; uint32_t m=0; while(m<258&&W[p+m]==W[q+m])m++; mbytes+=m; if(m>cl){cl=m; if(cl>=nice){nicestop++;break;}}}
            it++; d=p4[q]; q-=d; } }
    out[0]=hops/len; out[1]=pass/len; out[2]=mbytes/len; out[3]=nicestop/len; out[4]=full/len;
    free(p4);free(h4);free(W);
}
