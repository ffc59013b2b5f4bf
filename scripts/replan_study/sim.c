/* Hourly re-plan study (CPU only, test infrastructure):
 * counts, per lane-day and per 64-lane wave-day, the hours in which the exact
 * 24-hour target must be formed
 *   A  the hourly rule as the oracle states it (every hour that can discharge)
 *   B  a carried target: kept exact while no hour above it enters the window
 *      and no charge happens, else kept as a lower bound that decides "no
 *      discharge" hours without a re-plan
 * and checks that B's state of charge follows A's (rounding-level). */
#include "../../oracle/orc.c"
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>
static double clampd(double n, double T, double P, double av){double d=n-T; if(d<0)d=0; if(d>P)d=P; if(d>av)d=av; return d;}
int main(int argc,char**argv){
  int n=atoi(argv[1]); int NHh=8760;
  if(argc>2 && chdir(argv[2])!=0) return 1;
  double *L=malloc(8*n*NHh),*PV=malloc(8*n*NHh),*B=malloc(8*n),*P=malloc(8*n);
  FILE*f=fopen("load.bin","rb");fread(L,8,(size_t)n*NHh,f);fclose(f);
  f=fopen("pv.bin","rb");fread(PV,8,(size_t)n*NHh,f);fclose(f);
  f=fopen("bank.bin","rb");fread(B,8,n,f);fclose(f);
  f=fopen("power.bin","rb");fread(P,8,n,f);fclose(f);
  const double mn=0.10,mx=0.95,ei=0.9408,eo=0.9408,s0=0.30;
  unsigned char *needA=calloc((size_t)n*NHh,1),*needB=calloc((size_t)n*NHh,1);
  double maxdiff=0; long lrA=0,lrB=0;
  for(int i=0;i<n;i++){
    const double*ld=L+(size_t)i*NHh,*pv=PV+(size_t)i*NHh; double bank=B[i],pw=P[i];
    double socA=s0,socB=s0,lo=0,Tc=0; int exact=0;
    double inv_in=1.0/ei,inpb=ei/bank,outpb=1.0/(eo*bank);
    for(int h=0;h<NHh;h++){
      double nn=ld[h]-pv[h];
      /* A */
      { double g;
        if(nn<0){double room=(mx-socA)*bank*inv_in; if(room<0)room=0; double c=-nn; if(c>pw)c=pw; if(c>room)c=room; socA+=c*inpb; g=0;}
        else {double av=(socA-mn)*bank*eo; if(av<0)av=0; double T=0; if(nn>0&&av>0){T=day_target(ld,pv,h,pw,av); needA[(size_t)i*NHh+h]=1;}
              double d=clampd(nn,T,pw,av); socA-=d*outpb; g=nn-d;}
        (void)g;
      }
      /* B */
      { int hn=(h+24)%NHh; double dnew=ld[hn]-pv[hn]; if(dnew<0)dnew=0;
        if(nn<0){double room=(mx-socB)*bank*inv_in; if(room<0)room=0; double c=-nn; if(c>pw)c=pw; if(c>room)c=room; socB+=c*inpb;
                 if(c>0){lo=0;exact=0;} else if(exact && dnew>Tc){exact=0; lo=Tc;} }
        else {double av=(socB-mn)*bank*eo; if(av<0)av=0; double T=0;
              if(nn>0&&av>0){
                 if(exact) T=Tc;
                 else if(nn<=lo) T=lo;
                 else {T=day_target(ld,pv,h,pw,av); Tc=T; lo=T; exact=1; needB[(size_t)i*NHh+h]=1;}
                 double dun=nn-T; if(dun<0)dun=0; if(dun>pw)dun=pw;
                 double d=clampd(nn,T,pw,av);
                 if(exact){ if(T<=0 || d<dun){exact=0; lo=0;} else if(dnew>Tc){exact=0; lo=Tc;} }
                 socB-=d*outpb;
              } else if(nn>0){ lo=0; exact=0; }
              else { if(exact && dnew>Tc){exact=0; lo=Tc;} }
        }
      }
      double df=socA-socB; if(df<0)df=-df; if(df>maxdiff)maxdiff=df;
    }
  }
  long wA=0,wB=0,nw=0;
  for(int w=0;w+64<=n;w+=64){ for(int h=0;h<NHh;h++){int a=0,b=0; for(int k=0;k<64;k++){a|=needA[(size_t)(w+k)*NHh+h]; b|=needB[(size_t)(w+k)*NHh+h]; lrA+=needA[(size_t)(w+k)*NHh+h]; lrB+=needB[(size_t)(w+k)*NHh+h];} wA+=a; wB+=b;} nw++;}
  printf("lane refresh per lane-day: A %.2f B %.2f ; wave refresh-hours per day: A %.2f B %.2f ; max soc diff %.3g\n",
     lrA/(double)(nw*64)/365, lrB/(double)(nw*64)/365, wA/(double)nw/365, wB/(double)nw/365, maxdiff);
}
