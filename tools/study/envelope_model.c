// CPU model of the envelope solve: pass 0 walks every super-tile
// of U frames from a guess (the M of its first frame, or a warm-up walk of W frames),
// then fix-up sweeps as csrc/compressor.hip runs them — sweep 1 a Jacobi step
// without continuation, later sweeps from run heads with continuation — with
// exact release jumps over SEGL-frame segments whose every entry state exceeds
// their largest M (cost J steps), stopping at the first CMP-aligned frame where
// the walk meets the stored trajectory.  Prints per band the summed latency of the
// sweeps (the longest walk of each sweep) in step equivalents, and checks that the
// converged trajectory equals the true one.
// gcc -O2 -DSEGL=125 -DCMP=125 -o /tmp/em tools/study/envelope_model.c
// /tmp/em /tmp/study/full.idx 1000 0 [J]   (data: tools/study/envelope_data.py)
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
static double step(double a,double m,double A,double R){double inc=m/A,dec=m/R; if(a<=m){double u=a+inc;return u<m?u:m;} double d=a-dec; return d>0?d:0;}
static double *M,*smax; static long n; static double A_,R_,J;
// walk super-tile range [s,e) from state a, comparing with stored ck at 40-frame blocks; returns cost, sets *co, *out
static double walk(double a,long s,long e,double*st,int check,int*co,double*out){ double cost=0; long i=s; *co=0;
  while(i<e){ if(check && (i-s)%CMP==0 && st[i]==a){*co=1; return cost;}
    if(i%SEGL==0 && i+SEGL<=e && a>smax[i/SEGL]) { // jump (exact by construction in the real kernel): walk it for the value
      for(int k=0;k<SEGL;k++){st[i+k]=a; a=step(a,M[i+k],A_,R_);} i+=SEGL; cost+=J; continue; }
    st[i]=a; a=step(a,M[i],A_,R_); i++; cost+=1; }
  *out=a; return cost; }
int main(int argc,char**argv){
  FILE*f=fopen(argv[1],"r"); long U=atol(argv[2]); long W=atol(argv[3]); J=argc>4?atof(argv[4]):3;
  char path[256]; int b; double tot_lat[3]={0}; int cnt[3]={0}; double worst[3]={0}; int maxsw[3]={0};
  while(fscanf(f,"%s %d %ld %lf %lf",path,&b,&n,&A_,&R_)==5){
    M=malloc(n*8); FILE*g=fopen(path,"rb"); if(fread(M,8,n,g)!=(size_t)n) return 1; fclose(g);
    long nseg=n/SEGL+1; smax=calloc(nseg,8); for(long i=0;i<n;i++) if(M[i]>smax[i/SEGL]) smax[i/SEGL]=M[i];
    double*tr=malloc((n+1)*8); tr[0]=0; for(long i=0;i<n;i++) tr[i+1]=step(tr[i],M[i],A_,R_);
    long NS=(n+U-1)/U; double*st=malloc((n+1)*8),*start=malloc(NS*8),*end=malloc(NS*8);
    for(long s=0;s<NS;s++){ long p=s*U; double a; if(p==0)a=0; else { long w0=p-W; if(w0<=0){a=0;w0=0;} else a=M[w0]; for(long i=w0;i<p;i++) a=step(a,M[i],A_,R_);} 
      start[s]=a; long e=p+U<n?p+U:n; for(long i=p;i<e;i++){st[i]=a;a=step(a,M[i],A_,R_);} end[s]=a; }
    double lat=0; int sw;
    for(sw=1;sw<50;sw++){ double mx=0; int any=0; double*oldend=malloc(NS*8); memcpy(oldend,end,NS*8);
      char*claimed=calloc(NS,1);
      for(long s=1;s<NS;s++){ if(start[s]==oldend[s-1]) continue; any=1;
        if(sw>1 && s>1 && start[s-1]!=oldend[s-2]) continue; // inside a run
        if(claimed[s]) continue;
        double a=oldend[s-1], c=0; long cur=s;
        for(;;){ claimed[cur]=1; start[cur]=a; int co; double o; long p=cur*U,e=p+U<n?p+U:n;
          c+=walk(a,p,e,st,1,&co,&o); if(co) break; end[cur]=o; if(cur+1>=NS) break;
          if(sw==1) break; // Jacobi: successors claimed by their own lanes
          if(claimed[cur+1]) break; cur++; a=o; }
        if(c>mx) mx=c; }
      free(oldend); free(claimed); if(!any) break; lat+=mx; }
    // verify
    for(long i=0;i<n;i++) if(st[i]!=tr[i]) { printf("MISMATCH band %d at %ld\n",b,i); break; }
    tot_lat[b]+=lat; cnt[b]++; if(lat>worst[b]) worst[b]=lat; if(sw>maxsw[b]) maxsw[b]=sw;
    free(M);free(smax);free(tr);free(st);free(start);free(end);
  }
  for(b=0;b<3;b++) if(cnt[b]) printf("U=%ld W=%ld J=%.0f band %d: sweep latency mean %.0f max %.0f step-eq, sweeps(max) %d\n",U,W,J,b,tot_lat[b]/cnt[b],worst[b],maxsw[b]);
}
